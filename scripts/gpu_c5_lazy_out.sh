#!/bin/bash
# C5 on one GPU: the out table's Adam dense (fused into pass 2) vs lazy exact,
# plus the STREAM-copy variants. Logs under gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/microbench/copy_rates > gpurun_out/copy_rates.log 2>&1 || exit 1
cat gpurun_out/copy_rates.log
for lo in off on; do
  echo "=== c5 lazy-out $lo ($(date +%T))"
  timeout -k 10 400 python bench.py --config c5 --steps 60 --warmup 5 --no-cpu-baseline \
    --no-walk-bench --lazy-out $lo > gpurun_out/c5_lazy_out_$lo.log 2>&1 || { tail -5 gpurun_out/c5_lazy_out_$lo.log; exit 1; }
  tail -c 600 gpurun_out/c5_lazy_out_$lo.log
done
