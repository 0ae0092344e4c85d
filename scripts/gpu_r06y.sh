#!/bin/bash
# Round 6 A/B: k_out_rows' resident blocks per CU capped (DW_OUT_ROWS_CAP; 0 = every range its own
# block, 7 per CU resident) so that the in rows' catch-up beside it finds free wave slots — the
# steady state's bottleneck; batch64 at 400 steps and the last 4,000 of 20,000.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for c in 0 6 5 4; do
    DW_OUT_ROWS_CAP=$c timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 > gpurun_out/r06y_${c}_$r.log 2>&1 || { tail -5 gpurun_out/r06y_${c}_$r.log; exit 1; }
    grep '^{' gpurun_out/r06y_${c}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('cap $c', round(b['ms_per_step'],4), round(b['steady_state']['ms_per_step'],4), b['step_check']['ok'])"
  done
done
