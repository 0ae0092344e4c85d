#!/bin/bash
# node2vec walker: hashed adjacency vs sorted-list search, product build (8 waves/SIMD forced)
# vs an unconstrained-occupancy build; then the walker GPU tests.
set -u
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_walks.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/n2v_tests.log 2>&1; rc=$?; tail -3 gpurun_out/n2v_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/microbench/walk_rates.py --counts 65536,1048576 || exit 1
echo "=== wpe1"; DW_LIB_PATH=$PWD/scripts/debug/exp/libdw_hip_wpe1.so timeout -k 10 200 python scripts/microbench/walk_rates.py --counts 65536,1048576 || exit 1
echo "=== c5 graph"; timeout -k 10 300 python scripts/microbench/walk_rates.py --scale 24 --edges 268435456 --counts 65536,1048576 || exit 1
