#!/bin/bash
# C3 at 64 walks: the placed records and the p-only catch-up A/B (DW_OUT_PLACE, DW_OUT_P_ONLY),
# then a kernel trace of the default (scripts/gpu_trace_c3_64.sh). Logs under gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "1 1" "0 0" "1 0" "0 1" "1 1"; do
  set -- $cfg
  DW_OUT_PLACE=$1 DW_OUT_P_ONLY=$2 timeout -k 10 300 python bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench --exact-steps 0 > gpurun_out/c3_64_p$1_o$2.log 2>&1 || { tail -5 gpurun_out/c3_64_p$1_o$2.log; exit 1; }
  grep '^{' gpurun_out/c3_64_p$1_o$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('place', '$1', 'p_only', '$2', d['ms_per_step'])"
done
bash scripts/gpu_trace_c3_64.sh || exit 1
