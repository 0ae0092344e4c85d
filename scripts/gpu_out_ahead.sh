#!/bin/bash
# The next batch's out-row claim + catch-up beside the step before's output-table phase
# (OwnerLazyTables.catch_up_out_ahead): its tests, then C3 at 64 walks with DW_OUT_AHEAD 1 / 0 / 1.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_owner.py tests/test_gpu_graphed.py tests/test_gpu_c3_step.py -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread > gpurun_out/out_ahead_tests.log 2>&1; rc=$?
tail -6 gpurun_out/out_ahead_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for a in 1 0 1; do
  DW_OUT_AHEAD=$a timeout -k 10 300 python bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench > gpurun_out/c3_64_ahead$a.log 2>&1 || { tail -5 gpurun_out/c3_64_ahead$a.log; exit 1; }
  grep '^{' gpurun_out/c3_64_ahead$a.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('out_ahead $a', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
