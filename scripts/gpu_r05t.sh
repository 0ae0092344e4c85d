#!/bin/bash
# Round 5: k_out_rows with the next row's centre rows staged by LDS-DMA — the tests that run it,
# the 64-walk step (bench batch64 line) twice, and its kernel stats. Outputs gpurun_out/r05t_*.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_graphed.py tests/test_gpu_exact.py tests/test_gpu_owner.py > gpurun_out/r05t_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05t_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 > gpurun_out/r05t_bench$i.log 2>&1 || { tail -5 gpurun_out/r05t_bench$i.log; exit 1; }
  grep '^{' gpurun_out/r05t_bench$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('batch64', b['ms_per_step'], b['value'], b['roofline']['frac'], b['step_check']['ok'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05t_prof -o run --output-format csv -- python3 bench.py --batch-walks 64 --steps 32 --warmup 4 --no-cpu-baseline --no-walk-bench --exact-steps 0 --batch64-steps 0 > gpurun_out/r05t_prof.log 2>&1 || { tail -5 gpurun_out/r05t_prof.log; exit 1; }
f=$(find gpurun_out/r05t_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r05t_stats.csv
rm -rf gpurun_out/r05t_prof
head -8 gpurun_out/r05t_stats.csv | cut -d, -f1-4 | cut -c1-150
