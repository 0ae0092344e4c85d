#!/bin/bash
# Round 5: the walk tests (position walker), the bench with batch64 / walk rates, the N > 1
# flow rehearsed with the layout calibration (one nccl rank with DW_BENCH_DIST=1, two gloo ranks
# on the device), and the C5 position-index measurement. Logs under gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_walks.py tests/test_gpu_walk_law.py tests/test_gpu_graphed.py > gpurun_out/r05b_walk_tests.log 2>&1 || { tail -30 gpurun_out/r05b_walk_tests.log; exit 1; }
tail -2 gpurun_out/r05b_walk_tests.log
timeout -k 10 600 python bench.py --steps 40 --no-cpu-baseline > gpurun_out/r05b_bench.log 2>&1 || { tail -8 gpurun_out/r05b_bench.log; exit 1; }
grep '^{' gpurun_out/r05b_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('headline', d['value'], d['ms_per_step'], 'n2v walks/s', d['walks_per_s_node2vec_p0.25_q4'], d['roofline_walk']['node2vec']); print('batch64', b['value'], b['ms_per_step'], b['roofline']['frac'], b['roofline']['touched_in_rows'], b['roofline']['touched_out_rows'], b['step_check'])"
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 400 env DW_BENCH_DIST=1 $TR --nproc-per-node 1 --master-port 29611 bench.py --steps 20 --warmup 3 --no-walk-bench > gpurun_out/r05b_rccl_c3.log 2>&1 || { tail -20 gpurun_out/r05b_rccl_c3.log; exit 1; }
grep '^{' gpurun_out/r05b_rccl_c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rccl w1', d['layout'], d['layout_calibration_ms_per_step'], d['in_exchange_calibration_ms_per_step'], d['step_check']['ok'])"
timeout -k 10 400 env DW_BENCH_DIST=1 DW_BENCH_CORRUPT=1 $TR --nproc-per-node 1 --master-port 29612 bench.py --steps 4 --warmup 2 --no-walk-bench --dist-mode replicated > gpurun_out/r05b_rccl_repl_corrupt.log 2>&1; echo "replicated corrupt rc=$? (3 expected)"
timeout -k 10 400 env DW_BENCH_DIST=1 $TR --nproc-per-node 1 --master-port 29613 bench.py --steps 8 --warmup 2 --no-walk-bench --dist-mode replicated > gpurun_out/r05b_rccl_repl.log 2>&1 || { tail -20 gpurun_out/r05b_rccl_repl.log; exit 1; }
grep '^{' gpurun_out/r05b_rccl_repl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rccl w1 replicated', d['layout'], d['step_check'])"
timeout -k 10 400 env DW_BENCH_BACKEND=gloo DW_BENCH_ONE_DEVICE=1 $TR --nproc-per-node 2 --master-port 29614 bench.py --gpus 2 --steps 4 --warmup 1 --no-cpu-baseline --no-walk-bench --layout-calib on --calib-steps 2 > gpurun_out/r05b_gloo_w2.log 2>&1 || { tail -20 gpurun_out/r05b_gloo_w2.log; exit 1; }
grep '^{' gpurun_out/r05b_gloo_w2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('gloo w2', d['layout'], d['layout_calibration_ms_per_step'], d['step_check'])"
timeout -k 10 700 python -u scripts/microbench/n2v_index_c5.py > gpurun_out/r05b_n2v_c5.log 2>&1 || { tail -5 gpurun_out/r05b_n2v_c5.log; exit 1; }
cat gpurun_out/r05b_n2v_c5.log
