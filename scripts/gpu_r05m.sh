#!/bin/bash
# Round 5: the dense Adam's skipped zero stores — Adam / SGNS tests, then the headline line and
# the deterministic line at C3 (400 steps each).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_sgns.py tests/test_gpu_exact.py tests/test_gpu_c3_step.py > gpurun_out/r05m_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05m_tests.log; [ $rc -eq 0 ] || exit $rc
for m in float det; do
  extra=""; [ $m = det ] && extra="--deterministic"
  timeout -k 10 400 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-walk-bench --batch64-steps 0 $extra > gpurun_out/r05m_$m.log 2>&1 || { tail -5 gpurun_out/r05m_$m.log; exit 1; }
  grep '^{' gpurun_out/r05m_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', d['ms_per_step'], d['value'], d['roofline']['frac'])"
done
