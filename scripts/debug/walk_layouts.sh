#!/bin/bash
# Walkers: edge-inline layout (+ adjacency hash) vs plain CSR (+ sorted search): GPU walker
# tests, then rates on the C3 and C5 graphs (scripts/microbench/walk_rates.py).
set -u
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_walks.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/walk_tests.log 2>&1; rc=$?; tail -3 gpurun_out/walk_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/microbench/walk_rates.py --counts 8192,65536,1048576 || exit 1
echo "=== c5 graph"; timeout -k 10 300 python scripts/microbench/walk_rates.py --scale 24 --edges 268435456 --counts 8192,65536,1048576 || exit 1
