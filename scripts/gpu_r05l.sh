#!/bin/bash
# Round 5: the deterministic mode's cheaper conversion and centre atomics — exact tests, the
# C3 / 8,192 float vs deterministic kernel stats, the 64-walk deterministic line.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_exact.py tests/test_gpu_graphed.py > gpurun_out/r05l_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05l_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r05k.sh || exit 1
timeout -k 10 300 python bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench --deterministic > gpurun_out/r05l_c3_64_det.log 2>&1 || { tail -5 gpurun_out/r05l_c3_64_det.log; exit 1; }
grep '^{' gpurun_out/r05l_c3_64_det.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3/64 det', d['value'], d['ms_per_step'])"
