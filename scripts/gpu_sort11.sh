#!/bin/bash
# Small sorts of > 16 key bits on two 11-bit passes (DW_SORT_SMALL11=1) vs three 8-bit passes:
# the owner tests with the knob on, then C3 at 64 walks 0 / 1 / 0 / 1.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
DW_SORT_SMALL11=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_owner.py tests/test_gpu_graphed.py -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread > gpurun_out/sort11_tests.log 2>&1; rc=$?
tail -4 gpurun_out/sort11_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for a in 0 1 0 1; do
  DW_SORT_SMALL11=$a timeout -k 10 300 python bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench > gpurun_out/c3_64_sort11_$a.log 2>&1 || { tail -5 gpurun_out/c3_64_sort11_$a.log; exit 1; }
  grep '^{' gpurun_out/c3_64_sort11_$a.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('sort_small11 $a', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
