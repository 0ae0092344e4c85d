#!/bin/bash
# Round 6: batch64 with and without the frozen replay tails (A/B, interleaved), then the trace of
# each (the in-table catch-up's time).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for v in 0 1; do
    DW_NO_FREEZE=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 > gpurun_out/r06j_$v$i.log 2>&1 || { tail -5 gpurun_out/r06j_$v$i.log; exit 1; }
    grep '^{' gpurun_out/r06j_$v$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('no_freeze=$v', b['ms_per_step'], b['step_check']['ok'])"
  done
done
for v in 0 1; do
  DW_NO_FREEZE=$v bash scripts/gpu_prof_c3_64.sh > gpurun_out/r06j_prof$v.log 2>&1 || { tail -5 gpurun_out/r06j_prof$v.log; exit 1; }
  cp gpurun_out/prof64_kernel_trace.csv gpurun_out/r06j_trace$v.csv
  cp gpurun_out/prof64_kernel_stats.csv gpurun_out/r06j_stats$v.csv
done
