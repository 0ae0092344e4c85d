#!/bin/bash
# Round 6: the out rows captured before the next step's side chain (dispatch order) — parity of
# the pipelined / graphed steps, then batch64 three times and a trace.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_gpu_graphed.py "tests/test_gpu_exact.py::test_exact_lazy_rows_major_repeatable_and_equal_dense" \
  > gpurun_out/r06k_tests.log 2>&1 || { tail -40 gpurun_out/r06k_tests.log; exit 1; }
tail -1 gpurun_out/r06k_tests.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 > gpurun_out/r06k_$i.log 2>&1 || { tail -5 gpurun_out/r06k_$i.log; exit 1; }
  grep '^{' gpurun_out/r06k_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('batch64', b['ms_per_step'], b['step_check']['ok'])"
done
bash scripts/gpu_prof_c3_64.sh > gpurun_out/r06k_prof.log 2>&1 || { tail -5 gpurun_out/r06k_prof.log; exit 1; }
