#!/bin/bash
# Round-4 evidence on the final code, last pass: smoke, every GPU test, the default bench line,
# the batch shapes, and the 64-walk kernel trace. Logs under gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_check.sh || exit 1
BATCH_SPECS="c3_64:--batch-walks 64 --steps 400;c3_1024:--batch-walks 1024 --steps 100;c2:--config c2 --steps 400;c3_64_det:--batch-walks 64 --steps 200 --deterministic" bash scripts/gpu_batches.sh || exit 1
bash scripts/gpu_trace_c3_64.sh || exit 1
python3 scripts/trace_summary.py gpurun_out/trace64_kernel_trace.csv timeline > gpurun_out/r04_c3_64_trace.txt
tail -14 gpurun_out/r04_c3_64_trace.txt
