#!/bin/bash
# Round 6: batch64 with the frozen replay tail in the in-table catch-up only: two bench lines,
# then a kernel trace of the graphed 64-walk step.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_owner.py -k "long_lag or lazy" > gpurun_out/r06e_tests.log 2>&1 || { tail -30 gpurun_out/r06e_tests.log; exit 1; }
tail -1 gpurun_out/r06e_tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 > gpurun_out/r06e_b$i.log 2>&1 || { tail -5 gpurun_out/r06e_b$i.log; exit 1; }
  grep '^{' gpurun_out/r06e_b$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('headline', d['ms_per_step'], 'batch64', b['ms_per_step'], b['roofline']['frac'], b['step_check']['ok'])"
done
bash scripts/gpu_prof_c3_64.sh > gpurun_out/r06e_prof.log 2>&1 || { tail -5 gpurun_out/r06e_prof.log; exit 1; }
head -3 gpurun_out/r06e_prof.log
