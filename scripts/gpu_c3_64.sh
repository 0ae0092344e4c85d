#!/bin/bash
# C3 at the reference's 64-walk batch (one GPU, lazy in + out Adam, replayed as a HIP graph):
# graph on / off, then a kernel-stats profile and a kernel trace of the default. Logs under
# gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for g in auto off; do
  timeout -k 10 300 python bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench --graph $g > gpurun_out/c3_64_graph$g.log 2>&1 || { tail -5 gpurun_out/c3_64_graph$g.log; exit 1; }
  grep '^{' gpurun_out/c3_64_graph$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('graph $g', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof64 -o run --output-format csv -- python3 bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench > gpurun_out/prof64.log 2>&1 || { tail -5 gpurun_out/prof64.log; exit 1; }
find gpurun_out/prof64 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/prof64_kernel_stats.csv
rm -rf gpurun_out/prof64
bash scripts/gpu_trace_c3_64.sh
