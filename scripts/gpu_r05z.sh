#!/bin/bash
# Round 5: the deterministic mode's cost at C3 / 64 walks on the final code — the batch64 line
# (400 graphed steps) in float and in deterministic mode, interleaved twice.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for m in float det; do
    extra=""; [ $m = det ] && extra="--deterministic"
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 $extra > gpurun_out/r05z_$m$i.log 2>&1 || { tail -5 gpurun_out/r05z_$m$i.log; exit 1; }
    grep '^{' gpurun_out/r05z_$m$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('$m', 'batch64', b['ms_per_step'], b['value'], b.get('deterministic'), b['step_check']['ok'], 'headline', d['ms_per_step'])"
  done
done
