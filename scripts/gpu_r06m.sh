#!/bin/bash
# Round 6: whole rows per range in k_out_rows (no straddling rows, no boundary launch) — the
# rows-major parity tests (gather path with hub rows, no collisions, deterministic = dense,
# pipelined, graphed, full-size C3 at 64 walks, two ranks), then batch64 three times + a trace.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_gpu_owner.py tests/test_gpu_graphed.py tests/test_gpu_exact.py \
  "tests/test_gpu_c3_step.py" > gpurun_out/r06m_tests.log 2>&1 || { tail -40 gpurun_out/r06m_tests.log; exit 1; }
tail -1 gpurun_out/r06m_tests.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 > gpurun_out/r06m_$i.log 2>&1 || { tail -5 gpurun_out/r06m_$i.log; exit 1; }
  grep '^{' gpurun_out/r06m_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('batch64', round(b['ms_per_step'],4), b['step_check']['ok'])"
done
bash scripts/gpu_prof_c3_64.sh > gpurun_out/r06m_prof.log 2>&1 || { tail -5 gpurun_out/r06m_prof.log; exit 1; }
