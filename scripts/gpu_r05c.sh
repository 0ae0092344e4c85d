#!/bin/bash
# Round 5: kernel trace + SQ counters of the 64-walk C3 step (packed replays), and the C5
# position-index sizes with the wave walker's rate. Logs under gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_trace_c3_64.sh || exit 1
python3 scripts/trace_summary.py gpurun_out/trace64_kernel_trace.csv timeline > gpurun_out/r05c_c3_64_trace.txt
head -30 gpurun_out/r05c_c3_64_trace.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/r05c_sq -o run --output-format csv -- python3 bench.py --batch-walks 64 --steps 16 --warmup 4 --no-cpu-baseline --no-walk-bench --exact-steps 0 > gpurun_out/r05c_sq.log 2>&1 || { echo "sq pass failed"; tail -5 gpurun_out/r05c_sq.log; }
f=$(find gpurun_out/r05c_sq -name "*counter_collection.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/r05c_sq.csv; rm -rf gpurun_out/r05c_sq
timeout -k 10 700 python -u scripts/microbench/n2v_index_c5.py --check-walks 16384 > gpurun_out/r05c_n2v_c5.log 2>&1 || { tail -5 gpurun_out/r05c_n2v_c5.log; exit 1; }
cat gpurun_out/r05c_n2v_c5.log
