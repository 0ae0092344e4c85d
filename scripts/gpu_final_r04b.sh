#!/bin/bash
# Round-4 evidence, part 2: the RCCL protocol test after the owner_step fix, the headline profile
# (kernel trace/stats + PMC passes, summarised into profiles/ as r04) and the other batch shapes.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_rccl.py -q -p no:cacheprovider -rf --timeout 500 > gpurun_out/r04_rccl_tests.log 2>&1 || { tail -20 gpurun_out/r04_rccl_tests.log; exit 1; }
tail -1 gpurun_out/r04_rccl_tests.log
bash scripts/gpu_profile.sh || exit 1
python3 scripts/rocprof_summary.py r04 5734400 > gpurun_out/rocprof_summary_r04.log 2>&1 || { tail -5 gpurun_out/rocprof_summary_r04.log; exit 1; }
tail -5 gpurun_out/rocprof_summary_r04.log
mkdir -p gpurun_out/profiles && cp profiles/r04_* profiles/sgns_pmc.json gpurun_out/profiles/ 2>/dev/null
BATCH_SPECS="c3_64:--batch-walks 64 --steps 400;c3_1024:--batch-walks 1024 --steps 100;c2:--config c2 --steps 400;c3_64_det:--batch-walks 64 --steps 200 --deterministic" bash scripts/gpu_batches.sh
