#!/bin/bash
# Round 5: the exact position walker's serial picks run by run (no hand-over), the pipelined
# 64-walk step's fork point, the deterministic lazy path — tests, the C5 walker rates, the
# 64-walk line (float both forks, deterministic) + trace.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_graphed.py tests/test_gpu_exact.py tests/test_gpu_walks.py > gpurun_out/r05i_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05i_tests.log; [ $rc -eq 0 ] || exit $rc
for f in after before; do
  DW_PIPE_FORK=$f timeout -k 10 300 python bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench > gpurun_out/r05i_c3_64_$f.log 2>&1 || { tail -5 gpurun_out/r05i_c3_64_$f.log; exit 1; }
  grep '^{' gpurun_out/r05i_c3_64_$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3/64 fork=$f', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
timeout -k 10 300 python bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench --deterministic > gpurun_out/r05i_c3_64_det.log 2>&1 || { tail -5 gpurun_out/r05i_c3_64_det.log; exit 1; }
grep '^{' gpurun_out/r05i_c3_64_det.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3/64 det', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('step_check', {}).get('ok'))"
bash scripts/gpu_trace_c3_64.sh > /dev/null || exit 1
python3 scripts/trace_summary.py gpurun_out/trace64_kernel_trace.csv timeline > gpurun_out/r05i_c3_64_trace.txt
cut -c1-120 gpurun_out/r05i_c3_64_trace.txt | tail -24
timeout -k 10 600 python -u scripts/microbench/n2v_index_c5.py > gpurun_out/r05i_n2v_c5.jsonl 2> gpurun_out/r05i_n2v_c5.log
rc=$?; cut -c1-400 gpurun_out/r05i_n2v_c5.jsonl; tail -2 gpurun_out/r05i_n2v_c5.log; exit $rc
