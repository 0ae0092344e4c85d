#!/bin/bash
# Kernel trace (timestamps) of a short 64-walk C3 run: the sequence of one step's kernels,
# copies and fills. Output gpurun_out/trace64_kernel_trace.csv.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/trace64 -o run --output-format csv -- python3 bench.py --batch-walks 64 --steps 32 --warmup 4 --no-cpu-baseline --no-walk-bench ${BENCH_ARGS:-} > gpurun_out/trace64.log 2>&1 || { tail -5 gpurun_out/trace64.log; exit 1; }
find gpurun_out/trace64 -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} gpurun_out/trace64_kernel_trace.csv
find gpurun_out/trace64 -name "*memory_copy_trace.csv" | head -1 | xargs -I{} cp {} gpurun_out/trace64_memcpy_trace.csv
rm -rf gpurun_out/trace64
wc -l gpurun_out/trace64_*.csv
