#!/bin/bash
# Round 5: the C5 exact / Philox node2vec walks test (R-MAT 24 position index).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_c5_walks.py > gpurun_out/r05n_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r05n_tests.log; exit $rc
