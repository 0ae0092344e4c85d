#!/bin/bash
# Round 6: GraphedOwnerStep's side-first capture from SIDE_FIRST_FROM steps on — the graphed /
# pipelined / exact tests, then batch64 (400 steps and the steady state) twice.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_gpu_graphed.py tests/test_gpu_exact.py tests/test_gpu_bench.py tests/test_gpu_c3_step.py > gpurun_out/r06aa_tests.log 2>&1 || { tail -40 gpurun_out/r06aa_tests.log; exit 1; }
tail -1 gpurun_out/r06aa_tests.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 > gpurun_out/r06aa_$r.log 2>&1 || { tail -5 gpurun_out/r06aa_$r.log; exit 1; }
  grep '^{' gpurun_out/r06aa_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('batch64', round(b['ms_per_step'],4), round(b['steady_state']['ms_per_step'],4), b['step_check']['ok'])"
done
