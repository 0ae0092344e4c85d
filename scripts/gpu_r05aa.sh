#!/bin/bash
# Round 5: k_out_rows taking rows more than 8 steps behind first (experimental build,
# DW_LIB_PATH) — the tests that run it, then batch64 against the product build, interleaved.
# Usage: gpu_r05aa.sh <exp .so>
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
EXP=$PWD/$1
DW_LIB_PATH=$EXP timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_graphed.py tests/test_gpu_exact.py tests/test_gpu_owner.py > gpurun_out/r05aa_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05aa_tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag, lib ('' = product)
  ( if [ -n "$2" ]; then export DW_LIB_PATH=$2; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 > gpurun_out/r05aa_$1.log 2>&1 ) || { tail -5 gpurun_out/r05aa_$1.log; exit 1; }
  grep '^{' gpurun_out/r05aa_$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('$1', b['ms_per_step'], b['value'], b['step_check']['ok'])"
}
for i in 1 2 3; do
  run base$i "" && run lpt$i $EXP || exit 1
done
