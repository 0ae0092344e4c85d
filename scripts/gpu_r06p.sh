#!/bin/bash
# Round 6: long-lag out rows replayed by the placement (dw_sgns_owner_out_catch_up replay_lag)
# — the rows-major parity tests, then batch64 at DW_OUT_REPLAY_LAG 0 / 9 / 5 / 17 interleaved.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_gpu_exact.py tests/test_gpu_owner.py tests/test_gpu_graphed.py \
  tests/test_gpu_c3_step.py > gpurun_out/r06p_tests.log 2>&1 || { tail -40 gpurun_out/r06p_tests.log; exit 1; }
tail -1 gpurun_out/r06p_tests.log
for r in 1 2; do
  for lag in 0 9 5 17; do
    DW_OUT_REPLAY_LAG=$lag timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 > gpurun_out/r06p_${lag}_$r.log 2>&1 || { tail -5 gpurun_out/r06p_${lag}_$r.log; exit 1; }
    grep '^{' gpurun_out/r06p_${lag}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('lag $lag', round(b['ms_per_step'],4), b['step_check']['ok'])"
  done
done
