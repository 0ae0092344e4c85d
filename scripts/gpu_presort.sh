#!/bin/bash
# The presorted lazy step: its tests (owner, graphed, C3 full-size step incl. lazy-out), then C3 at
# 64 walks with DW_PRESORT 1 / 0 (graph on), and a kernel trace of the default. Logs in gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_walks.py tests/test_gpu_owner.py tests/test_gpu_graphed.py tests/test_gpu_c3_step.py tests/test_gpu_trainer.py tests/test_gpu_sgns.py -q -p no:cacheprovider -rf --timeout 600 > gpurun_out/presort_tests.log 2>&1; rc=$?
tail -6 gpurun_out/presort_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for ps in 1 0; do
  DW_PRESORT=$ps timeout -k 10 300 python bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench > gpurun_out/c3_64_presort$ps.log 2>&1 || { tail -5 gpurun_out/c3_64_presort$ps.log; exit 1; }
  grep '^{' gpurun_out/c3_64_presort$ps.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('presort $ps', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
bash scripts/gpu_trace_c3_64.sh
