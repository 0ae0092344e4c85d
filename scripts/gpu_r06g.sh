#!/bin/bash
# Round 6: batch64 with the preparation chains on one or two side streams and the placement forked
# after the out rows or at the step start (A/B, interleaved twice).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for v in 00 10 01 11; do
    DW_PIPE_ONE_SIDE=${v:0:1} DW_PIPE_OUT_EARLY=${v:1:1} timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 > gpurun_out/r06g_$v$i.log 2>&1 || { tail -5 gpurun_out/r06g_$v$i.log; exit 1; }
    grep '^{' gpurun_out/r06g_$v$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('one_side/out_early=$v', b['ms_per_step'], b['step_check']['ok'])"
  done
done
