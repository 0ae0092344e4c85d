#!/bin/bash
# Round 6: the batch64 steady-state leg (bench.py --batch64-long) — the bench tests, then the
# default bench line. Logs gpurun_out/r06w_*.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bench.py > gpurun_out/r06w_tests.log 2>&1 || { tail -30 gpurun_out/r06w_tests.log; exit 1; }
tail -1 gpurun_out/r06w_tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/r06w_bench.log 2>&1 || { tail -10 gpurun_out/r06w_bench.log; exit 1; }
grep '^{' gpurun_out/r06w_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print(d['value'], d['ms_per_step'], b['ms_per_step'], b['steady_state'], b['step_check']['ok'], d['c5']['ms_per_step'])"
