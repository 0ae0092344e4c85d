#!/bin/bash
# Round 5: bench.py's flows as tests (the lazy owner step through owner_lazy_step), then the
# 64-walk C3 batch and its kernel trace. Logs in gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_bench.py > gpurun_out/r05f_tests.log 2>&1 || { tail -40 gpurun_out/r05f_tests.log; exit 1; }
tail -2 gpurun_out/r05f_tests.log
timeout -k 10 300 python bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench > gpurun_out/r05f_c3_64.log 2>&1 || { tail -5 gpurun_out/r05f_c3_64.log; exit 1; }
grep '^{' gpurun_out/r05f_c3_64.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3/64', d['value'], d['ms_per_step'], d['roofline']['frac'])"
bash scripts/gpu_trace_c3_64.sh > /dev/null || exit 1
python3 scripts/trace_summary.py gpurun_out/trace64_kernel_trace.csv timeline > gpurun_out/r05f_c3_64_trace.txt
cat gpurun_out/r05f_c3_64_trace.txt | cut -c1-120
