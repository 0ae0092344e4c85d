#!/bin/bash
# Kernel trace of the reference's 64-walk batch on C3 (one GPU, lazy in + out Adam): where a
# step's time goes (kernels vs gaps). Outputs under gpurun_out/prof64*.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --batch-walks 64 --steps 200 --no-cpu-baseline --no-walk-bench ${BENCH_ARGS:-} > gpurun_out/prof64_plain.log 2>&1 || { tail -5 gpurun_out/prof64_plain.log; exit 1; }
grep '^{' gpurun_out/prof64_plain.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('plain', d['ms_per_step'], d['kernel_ms'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof64 -o run --output-format csv -- python3 bench.py --batch-walks 64 --steps 200 --no-cpu-baseline --no-walk-bench ${BENCH_ARGS:-} > gpurun_out/prof64.log 2>&1 || { tail -5 gpurun_out/prof64.log; exit 1; }
find gpurun_out/prof64 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/prof64_kernel_stats.csv
find gpurun_out/prof64 -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} gpurun_out/prof64_kernel_trace.csv
rm -rf gpurun_out/prof64
head -30 gpurun_out/prof64_kernel_stats.csv
