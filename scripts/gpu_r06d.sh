#!/bin/bash
# Round 6: the frozen replay tail (bit-exact long lags), the lazy / pipelined / graphed / N > 1
# tests, the full-size C3 steps, then the bench line twice.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread \
  tests/test_gpu_owner.py tests/test_gpu_graphed.py tests/test_gpu_exact.py tests/test_gpu_c3_step.py \
  > gpurun_out/r06d_tests.log 2>&1 || { tail -40 gpurun_out/r06d_tests.log; exit 1; }
grep -E "replay .* ms|passed|failed" gpurun_out/r06d_tests.log | tail -8
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 > gpurun_out/r06d_b$i.log 2>&1 || { tail -5 gpurun_out/r06d_b$i.log; exit 1; }
  grep '^{' gpurun_out/r06d_b$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('headline', d['ms_per_step'], 'batch64', b['ms_per_step'], b['roofline']['frac'], b['step_check']['ok'])"
done
