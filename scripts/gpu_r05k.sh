#!/bin/bash
# Round 5: the deterministic mode's cost at C3 / 8,192 walks — kernel stats of the float and
# the deterministic step (dense path), 10 steps each. Outputs gpurun_out/r05k_*.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in float det; do
  extra=""; [ $m = det ] && extra="--deterministic"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r05k_$m -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-walk-bench --batch64-steps 0 $extra > gpurun_out/r05k_$m.log 2>&1 || { echo "$m failed"; tail -5 gpurun_out/r05k_$m.log; exit 1; }
  f=$(find gpurun_out/r05k_$m -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r05k_${m}_stats.csv
  f=$(find gpurun_out/r05k_$m -name "*kernel_trace.csv" | head -1); cp "$f" gpurun_out/r05k_${m}_trace.csv
  rm -rf gpurun_out/r05k_$m
  grep '^{' gpurun_out/r05k_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', d['ms_per_step'], d['value'])"
  head -12 gpurun_out/r05k_${m}_stats.csv | cut -d, -f1-4 | cut -c1-150
done
