#!/bin/bash
# Round 5: the compact (uint16 / int32) node2vec position index and the pipelined 64-walk step —
# walk and graph tests, the C5 (R-MAT 24) index build and walker rates, the 64-walk bench line and
# its kernel trace. Logs in gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_graphed.py tests/test_gpu_walks.py tests/test_gpu_walk_law.py > gpurun_out/r05h_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r05h_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench > gpurun_out/r05h_c3_64.log 2>&1 || { tail -5 gpurun_out/r05h_c3_64.log; exit 1; }
grep '^{' gpurun_out/r05h_c3_64.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3/64', d['value'], d['ms_per_step'], d['roofline']['frac'])"
bash scripts/gpu_trace_c3_64.sh > /dev/null || exit 1
python3 scripts/trace_summary.py gpurun_out/trace64_kernel_trace.csv timeline > gpurun_out/r05h_c3_64_trace.txt
cut -c1-120 gpurun_out/r05h_c3_64_trace.txt | tail -30
timeout -k 10 600 python -u scripts/microbench/n2v_index_c5.py > gpurun_out/r05h_n2v_c5.jsonl 2> gpurun_out/r05h_n2v_c5.log
rc=$?; cat gpurun_out/r05h_n2v_c5.jsonl; tail -3 gpurun_out/r05h_n2v_c5.log; exit $rc
