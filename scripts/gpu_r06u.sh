#!/bin/bash
# Round 6: the frozen replay tails with the history's constant betas (no per-step loads; v alone
# once m is +0) — the long-lag bit-exactness tests and the lazy-path suites, then batch64 at
# 400 and at 20,000 graph-replayed steps (the in rows' lags grow with the run: steady state).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread \
  tests/test_gpu_owner.py tests/test_gpu_exact.py tests/test_gpu_graphed.py \
  tests/test_gpu_c3_step.py > gpurun_out/r06u_tests.log 2>&1 || { tail -40 gpurun_out/r06u_tests.log; exit 1; }
tail -1 gpurun_out/r06u_tests.log
grep -E "replay .* ms|per-step betas" gpurun_out/r06u_tests.log | head -8
for n in 400 20000; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 --batch64-steps $n > gpurun_out/r06u_b64_$n.log 2>&1 || { tail -5 gpurun_out/r06u_b64_$n.log; exit 1; }
  grep '^{' gpurun_out/r06u_b64_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('batch64 $n steps', round(b['ms_per_step'],4), b['step_check']['ok'])"
done
