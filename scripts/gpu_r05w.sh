#!/bin/bash
# Round 5, final code: the whole -m gpu suite, smoke(), the default bench line (headline +
# batch64 + walk rates + CPU baseline), and a kernel trace of the 64-walk step.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05w_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05w_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05w_smoke.log 2>&1 || { tail -5 gpurun_out/r05w_smoke.log; exit 1; }
tail -2 gpurun_out/r05w_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r05w_bench.log 2>&1 || { tail -5 gpurun_out/r05w_bench.log; exit 1; }
grep '^{' gpurun_out/r05w_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('headline', d['value'], d['ms_per_step'], d['roofline']['frac'], 'n2v', d['walks_per_s_node2vec_p0.25_q4']); print('batch64', b['value'], b['ms_per_step'], b['roofline']['frac'], b['step_check']['ok'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05w_prof -o run --output-format csv -- python3 bench.py --batch-walks 64 --steps 32 --warmup 4 --no-cpu-baseline --no-walk-bench --exact-steps 0 --batch64-steps 0 > gpurun_out/r05w_prof.log 2>&1 || { tail -5 gpurun_out/r05w_prof.log; exit 1; }
f=$(find gpurun_out/r05w_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r05w_c3_64_stats.csv
rm -rf gpurun_out/r05w_prof
echo done
