#!/bin/bash
# C3 at 64 walks: the placed records and the p-only catch-up A/B (DW_OUT_PLACE, DW_OUT_P_ONLY),
# then a kernel trace of the default (scripts/gpu_trace_c3_64.sh). Logs under gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "1 1" "0 0" "1 0" "0 1" "1 1"; do
  set -- $cfg
  DW_OUT_PLACE=$1 DW_OUT_P_ONLY=$2 timeout -k 10 300 python bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench --exact-steps 0 > gpurun_out/c3_64_p$1_o$2.log 2>&1 || { tail -5 gpurun_out/c3_64_p$1_o$2.log; exit 1; }
  grep '^{' gpurun_out/c3_64_p$1_o$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('place', '$1', 'p_only', '$2', d['ms_per_step'])"
done
bash scripts/gpu_trace_c3_64.sh || exit 1
# the node2vec position index: parity tests, then the walk bench (replay stats)
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_walks.py -k "n2v_position or indexed_node2vec or edge_counts_same or hubs or self_looped" > gpurun_out/r04b_n2v_tests.log 2>&1 || { tail -40 gpurun_out/r04b_n2v_tests.log; exit 1; }
tail -3 gpurun_out/r04b_n2v_tests.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --exact-steps 0 > gpurun_out/r04b_walkbench.log 2>&1 || { tail -20 gpurun_out/r04b_walkbench.log; exit 1; }
grep '^{' gpurun_out/r04b_walkbench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({k: d.get(k) for k in ('walks_per_s_replay','roofline_walk')}, indent=1))"
# the deterministic mode (tests/test_gpu_exact.py); a plain test failure (rc 1) does not stop the script
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_exact.py > gpurun_out/r04b_exact_tests.log 2>&1
rc=$?
tail -25 gpurun_out/r04b_exact_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
# the deterministic mode's cost: C3 (8192 walks) and C3/64 (dense in-table Adam, records), float vs exact
for b in 8192 64; do
  for det in "" "--deterministic"; do
    tag=det_b${b}${det:+_exact}
    timeout -k 10 300 python bench.py --batch-walks $b --steps 100 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 --n1-in-adam dense --scatter sorted $det > gpurun_out/$tag.log 2>&1 || { tail -5 gpurun_out/$tag.log; exit 1; }
    grep '^{' gpurun_out/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['ms_per_step'], d.get('deterministic'))"
  done
done
# the records sort's tile / digit configurations
timeout -k 10 180 ./scripts/microbench/sort_bench > gpurun_out/r04b_sort_bench.txt 2>&1 || { tail -5 gpurun_out/r04b_sort_bench.txt; exit 1; }
cat gpurun_out/r04b_sort_bench.txt
