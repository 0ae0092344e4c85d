#!/bin/bash
# Round 5: kernel trace of the C3 / 8,192 step with the lazy in-table Adam (timeline of a step).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r05s -o run --output-format csv -- python3 bench.py --steps 12 --warmup 2 --no-cpu-baseline --no-walk-bench --batch64-steps 0 --exact-steps 0 --n1-in-adam lazy > gpurun_out/r05s.log 2>&1 || { tail -5 gpurun_out/r05s.log; exit 1; }
find gpurun_out/r05s -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} gpurun_out/r05s_trace.csv
rm -rf gpurun_out/r05s
python3 scripts/trace_summary.py gpurun_out/r05s_trace.csv timeline > gpurun_out/r05s_timeline.txt
cut -c1-120 gpurun_out/r05s_timeline.txt | tail -40
