#!/bin/bash
# Round 5: the counts cleared by the placement scan — owner / graphed / exact / C3 step tests,
# the 64-walk line, its trace and its FETCH / WRITE counters.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_owner.py tests/test_gpu_graphed.py tests/test_gpu_exact.py tests/test_gpu_c3_step.py tests/test_gpu_bench.py > gpurun_out/r05o_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05o_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench > gpurun_out/r05o_c3_64.log 2>&1 || { tail -5 gpurun_out/r05o_c3_64.log; exit 1; }
grep '^{' gpurun_out/r05o_c3_64.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3/64', d['value'], d['ms_per_step'], d['roofline']['frac'])"
bash scripts/gpu_trace_c3_64.sh > /dev/null || exit 1
python3 scripts/trace_summary.py gpurun_out/trace64_kernel_trace.csv timeline > gpurun_out/r05o_c3_64_trace.txt
cut -c1-120 gpurun_out/r05o_c3_64_trace.txt | tail -16
B="python3 bench.py --batch-walks 64 --steps 16 --warmup 4 --no-cpu-baseline --no-walk-bench --exact-steps 0"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/r05o_$c -o run --output-format csv -- $B > gpurun_out/r05o_$c.log 2>&1 || { echo "$c failed"; tail -3 gpurun_out/r05o_$c.log; exit 1; }
  f=$(find gpurun_out/r05o_$c -name "*counter_collection.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/r05o_$c.csv; rm -rf gpurun_out/r05o_$c
done
echo pmc done
