#!/bin/bash
# The lazy owner step as a HIP graph: its tests, then C3 at the reference's 64-walk batch with the
# graph off / on, then a kernel trace of the graphed run. Logs under gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_graphed.py tests/test_gpu_owner.py tests/test_gpu_c3_step.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/graph_owner_tests.log 2>&1; rc=$?
tail -5 gpurun_out/graph_owner_tests.log
[ $rc -eq 0 ] || exit $rc
for g in off on; do
  timeout -k 10 300 python bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench --graph $g > gpurun_out/c3_64_graph_$g.log 2>&1 || { tail -5 gpurun_out/c3_64_graph_$g.log; exit 1; }
  grep '^{' gpurun_out/c3_64_graph_$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('graph $g', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof64 -o run --output-format csv -- python3 bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench > gpurun_out/prof64.log 2>&1 || { tail -5 gpurun_out/prof64.log; exit 1; }
find gpurun_out/prof64 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/prof64_kernel_stats.csv
rm -rf gpurun_out/prof64
head -25 gpurun_out/prof64_kernel_stats.csv | cut -c1-200
