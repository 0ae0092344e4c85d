#!/bin/bash
# Round-5 evidence: the trainer / graphed tests touched last, then the headline profile (kernel
# trace / stats + FETCH / WRITE / atomic PMC passes, summarised into profiles/ as r05 by
# scripts/rocprof_summary.py). Logs under gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
true

BENCH_ARGS="--batch64-steps 0 ${BENCH_ARGS:-}" bash scripts/gpu_profile.sh || exit 1
python3 scripts/rocprof_summary.py r05 5734400 > gpurun_out/rocprof_summary_r05.log 2>&1 || { tail -5 gpurun_out/rocprof_summary_r05.log; exit 1; }
tail -5 gpurun_out/rocprof_summary_r05.log
mkdir -p gpurun_out/profiles && cp profiles/r05_kernel_stats.csv profiles/r05_pmc.json profiles/sgns_pmc.json gpurun_out/profiles/ 2>/dev/null
echo done
