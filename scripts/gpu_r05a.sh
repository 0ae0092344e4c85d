#!/bin/bash
# Round 5, first GPU call: the new / changed tests (d=192 lazy-owner fallback, accumulator
# registry, Philox position walker + laws), the bench with batch64 and the walk rates, and the
# C5 position-index measurement. Logs under gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_owner.py tests/test_gpu_exact.py tests/test_gpu_c3_step.py -k "registry or unbuilt_width or rows_major or lazy_single_rank or reciprocal or replay or lazy_out" > gpurun_out/r05a_tests.log 2>&1 || { tail -30 gpurun_out/r05a_tests.log; exit 1; }
tail -2 gpurun_out/r05a_tests.log
timeout -k 10 900 $T tests/test_gpu_walks.py tests/test_gpu_walk_law.py tests/test_gpu_graphed.py > gpurun_out/r05a_walk_tests.log 2>&1 || { tail -30 gpurun_out/r05a_walk_tests.log; exit 1; }
tail -2 gpurun_out/r05a_walk_tests.log
timeout -k 10 600 python bench.py --steps 40 --no-cpu-baseline > gpurun_out/r05a_bench.log 2>&1 || { tail -8 gpurun_out/r05a_bench.log; exit 1; }
grep '^{' gpurun_out/r05a_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('headline', d['value'], d['ms_per_step'], 'n2v walks/s', d['walks_per_s_node2vec_p0.25_q4'], d['roofline_walk']['node2vec']); print('batch64', b['value'], b['ms_per_step'], b['roofline']['frac'], b['roofline']['touched_in_rows'], b['roofline']['touched_out_rows'], b['step_check'])"
timeout -k 10 700 python -u scripts/microbench/n2v_index_c5.py > gpurun_out/r05a_n2v_c5.log 2>&1 || { tail -5 gpurun_out/r05a_n2v_c5.log; exit 1; }
cat gpurun_out/r05a_n2v_c5.log
