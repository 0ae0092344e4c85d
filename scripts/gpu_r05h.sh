#!/bin/bash
# Round 5: the compact (uint16 / int32) node2vec position index — walk tests, then the C5
# (R-MAT 24) index build and walker rates. Logs in gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_walks.py tests/test_gpu_walk_law.py > gpurun_out/r05h_walk_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r05h_walk_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/microbench/n2v_index_c5.py > gpurun_out/r05h_n2v_c5.jsonl 2> gpurun_out/r05h_n2v_c5.log
rc=$?; cat gpurun_out/r05h_n2v_c5.jsonl; tail -3 gpurun_out/r05h_n2v_c5.log; exit $rc
