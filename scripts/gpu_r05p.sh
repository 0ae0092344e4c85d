#!/bin/bash
# Round 5: where the one-GPU in-table Adam runs (beside the sort + gather, capped grid; or at
# full rate beside the sort only) — the C3 step test both ways, then the headline both ways.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
DW_ADAM_WINDOW=sort timeout -k 10 600 $T tests/test_gpu_c3_step.py -k "dense" > gpurun_out/r05p_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05p_tests.log; [ $rc -eq 0 ] || exit $rc
for w in pass2 sort pass2 sort; do
  DW_ADAM_WINDOW=$w timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-walk-bench --batch64-steps 0 --exact-steps 0 > gpurun_out/r05p_$w.log 2>&1 || { tail -5 gpurun_out/r05p_$w.log; exit 1; }
  grep '^{' gpurun_out/r05p_$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w', d['ms_per_step'], d['value'])"
done
