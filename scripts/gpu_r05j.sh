#!/bin/bash
# Round 5: the serial picks by binades — walk tests, the C5 walker rates, then the
# deterministic mode's cost at C3 / 8,192 (kernel stats, float vs deterministic).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_walks.py -k "positions or n2v or serial" > gpurun_out/r05j_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05j_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/microbench/n2v_index_c5.py > gpurun_out/r05j_n2v_c5.jsonl 2> gpurun_out/r05j_n2v_c5.log
rc=$?; cut -c1-400 gpurun_out/r05j_n2v_c5.jsonl | tail -4; tail -2 gpurun_out/r05j_n2v_c5.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r05k.sh
