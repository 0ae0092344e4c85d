#!/bin/bash
# Round 5: the C3 / 8,192 step with the lazy exact in-table Adam (owner path on one rank) vs the
# dense default, 200 steps each, twice.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for a in dense lazy dense lazy; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-walk-bench --batch64-steps 0 --exact-steps 0 --n1-in-adam $a > gpurun_out/r05r_$a.log 2>&1 || { tail -5 gpurun_out/r05r_$a.log; exit 1; }
  grep '^{' gpurun_out/r05r_$a.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$a', d['ms_per_step'], d['value'], d['config']['parallelism'][:60])"
done
