#!/bin/bash
# Round-6 evidence, part 2: the headline profile (kernel trace / stats + FETCH / WRITE / atomic
# PMC passes, summarised into profiles/ as r06 by scripts/rocprof_summary.py), then the 64-walk
# step's kernel trace (gpurun_out/prof64_kernel_stats.csv -> profiles/r06_c3_64_kernel_stats.csv).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
BENCH_ARGS="--batch64-steps 0 --c5-steps 0 ${BENCH_ARGS:-}" bash scripts/gpu_profile.sh || exit 1
python3 scripts/rocprof_summary.py r06 5734400 > gpurun_out/rocprof_summary_r06.log 2>&1 || { tail -5 gpurun_out/rocprof_summary_r06.log; exit 1; }
tail -5 gpurun_out/rocprof_summary_r06.log
mkdir -p gpurun_out/profiles && cp profiles/r06_kernel_stats.csv profiles/r06_pmc.json profiles/sgns_pmc.json gpurun_out/profiles/ || exit 1
bash scripts/gpu_prof_c3_64.sh > gpurun_out/r06_prof64.log 2>&1 || { tail -5 gpurun_out/r06_prof64.log; exit 1; }
echo done
