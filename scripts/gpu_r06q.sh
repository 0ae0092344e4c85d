#!/bin/bash
# Round 6 A/B: where the main stream joins step k + 1's preparation — at step k + 1's start
# (start, the committed form) or before step k's centre pass (early) — batch64 interleaved, then
# a kernel trace of the early form (the step-boundary gap).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_graphed.py tests/test_gpu_exact.py -k "pipelined or graphed_owner" > gpurun_out/r06q_tests.log 2>&1 || { tail -30 gpurun_out/r06q_tests.log; exit 1; }
DW_PIPE_JOIN=early timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_graphed.py tests/test_gpu_exact.py -k "pipelined or graphed_owner" >> gpurun_out/r06q_tests.log 2>&1 || { tail -30 gpurun_out/r06q_tests.log; exit 1; }
grep passed gpurun_out/r06q_tests.log
for r in 1 2 3; do
  for j in start early; do
    DW_PIPE_JOIN=$j timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 > gpurun_out/r06q_${j}_$r.log 2>&1 || { tail -5 gpurun_out/r06q_${j}_$r.log; exit 1; }
    grep '^{' gpurun_out/r06q_${j}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('join $j', round(b['ms_per_step'],4), b['step_check']['ok'])"
  done
done
DW_PIPE_JOIN=early bash scripts/gpu_prof_c3_64.sh > gpurun_out/r06q_prof.log 2>&1 || { tail -5 gpurun_out/r06q_prof.log; exit 1; }
