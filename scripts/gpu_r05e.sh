#!/bin/bash
# Round 5: the pending p-step + pipelined k_out_rows — the lazy / rows-major / exact / C3-step
# tests, then the 64-walk batch (bench batch64 line) and its kernel trace. Logs in gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_owner.py tests/test_gpu_graphed.py tests/test_gpu_c3_step.py tests/test_gpu_exact.py tests/test_gpu_c5_step.py > gpurun_out/r05e_tests.log 2>&1 || { tail -40 gpurun_out/r05e_tests.log; exit 1; }
tail -2 gpurun_out/r05e_tests.log
timeout -k 10 300 python bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench > gpurun_out/r05e_c3_64.log 2>&1 || { tail -5 gpurun_out/r05e_c3_64.log; exit 1; }
grep '^{' gpurun_out/r05e_c3_64.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3/64', d['value'], d['ms_per_step'], d['roofline']['frac'])"
bash scripts/gpu_trace_c3_64.sh > /dev/null || exit 1
python3 scripts/trace_summary.py gpurun_out/trace64_kernel_trace.csv timeline > gpurun_out/r05e_c3_64_trace.txt
head -16 gpurun_out/r05e_c3_64_trace.txt
