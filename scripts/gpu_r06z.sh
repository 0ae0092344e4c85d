#!/bin/bash
# Round 6 A/B at the steady state: step k + 1's preparation captured before step k's out rows
# (DW_SIDE_FIRST=1: the in-row catch-up dispatched first) against after (the committed order).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for sf in 0 1; do
    DW_SIDE_FIRST=$sf timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 > gpurun_out/r06z_${sf}_$r.log 2>&1 || { tail -5 gpurun_out/r06z_${sf}_$r.log; exit 1; }
    grep '^{' gpurun_out/r06z_${sf}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('side_first $sf', round(b['ms_per_step'],4), round(b['steady_state']['ms_per_step'],4), b['step_check']['ok'])"
  done
done
