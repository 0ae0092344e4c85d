#!/bin/bash
# The headline step with the records presorted ahead of pass 1 (DW_PRESORT_STEP=1): its parity
# tests, then bench.py's default C3 line with DW_PRESORT_STEP 0 / 1 / 0. Logs in gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sgns.py tests/test_gpu_graphed.py tests/test_gpu_c3_step.py -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread > gpurun_out/presort_step_tests.log 2>&1; rc=$?
tail -6 gpurun_out/presort_step_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for ps in 0 1 0; do
  DW_PRESORT_STEP=$ps timeout -k 10 300 python bench.py --no-cpu-baseline --no-walk-bench > gpurun_out/presort_step$ps.log 2>&1 || { tail -5 gpurun_out/presort_step$ps.log; exit 1; }
  grep '^{' gpurun_out/presort_step$ps.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('presort_step $ps', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
