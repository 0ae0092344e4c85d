#!/bin/bash
# Round 5: the exhaustive reciprocal-division proof and SQ counters of the 64-walk
# step's kernels. Logs in gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/microbench/div_proof.py > gpurun_out/r05g_div_proof.jsonl 2> gpurun_out/r05g_div_proof.log || { echo "div proof rc=$?"; tail -3 gpurun_out/r05g_div_proof.log; }
cat gpurun_out/r05g_div_proof.jsonl
B="python3 bench.py --batch-walks 64 --steps 16 --warmup 4 --no-cpu-baseline --no-walk-bench --exact-steps 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -d gpurun_out/r05g_sq1 -o run --output-format csv -- $B > gpurun_out/r05g_sq1.log 2>&1 || { echo "sq1 failed"; tail -3 gpurun_out/r05g_sq1.log; }
f=$(find gpurun_out/r05g_sq1 -name "*counter_collection.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/r05g_sq1.csv; rm -rf gpurun_out/r05g_sq1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES -d gpurun_out/r05g_sq2 -o run --output-format csv -- $B > gpurun_out/r05g_sq2.log 2>&1 || { echo "sq2 failed"; tail -3 gpurun_out/r05g_sq2.log; }
f=$(find gpurun_out/r05g_sq2 -name "*counter_collection.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/r05g_sq2.csv; rm -rf gpurun_out/r05g_sq2
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/r05g_$c -o run --output-format csv -- $B > gpurun_out/r05g_$c.log 2>&1 || { echo "$c failed"; tail -3 gpurun_out/r05g_$c.log; }
  f=$(find gpurun_out/r05g_$c -name "*counter_collection.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/r05g_$c.csv; rm -rf gpurun_out/r05g_$c
done
ls gpurun_out | grep r05g
