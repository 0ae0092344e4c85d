#!/bin/bash
# Round 4: C3 at 64 walks — the next batch's catch-up beside this step's gather, with the
# catch-up's grid capped (DW_ROWS_ADAM_GRID) so the gather keeps its waves; the fast division
# check; the owner / graphed / exact / trainer tests; the RCCL self-check.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 3 "gpurun_out/$name.log" | cut -c1-400
  return $rc
}
for cfg in "0 0" "1 1024" "1 512" "1 2048" "1 256" "0 0"; do
  set -- $cfg
  if [ "$2" = "0" ]; then unset DW_ROWS_ADAM_GRID; else export DW_ROWS_ADAM_GRID=$2; fi
  DW_OUT_AHEAD=$1 run r04d_c3_64_a$1_g$2 300 python bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench --exact-steps 0 || exit 1
  grep '^{' gpurun_out/r04d_c3_64_a$1_g$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ahead $1 grid $2', d['ms_per_step'])"
done
unset DW_ROWS_ADAM_GRID
timeout -k 10 120 ./scripts/microbench/div_check 200000 65536 0.999 > gpurun_out/r04d_div_check.txt 2>&1; echo "div_check rc=$?"; cat gpurun_out/r04d_div_check.txt
timeout -k 10 120 ./scripts/microbench/div_check 20000 65536 0.99 >> gpurun_out/r04d_div_check.txt 2>&1; echo "div_check rc=$?"; tail -1 gpurun_out/r04d_div_check.txt
run r04d_owner_graphed_tests 900 python -u -m pytest tests/test_gpu_owner.py tests/test_gpu_graphed.py -x -q -p no:cacheprovider -rf --timeout 600 --timeout-method thread
run r04d_exact_loop 600 python -u -m pytest tests/test_gpu_exact.py -x -q -p no:cacheprovider -rf --timeout 500 --timeout-method thread -k train_loop
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
DW_BENCH_DIST=1 run r04_rccl_check 300 $TR --master-port 29621 bench.py --steps 20 --warmup 3 --no-walk-bench --no-cpu-baseline || exit 1
DW_BENCH_DIST=1 DW_BENCH_CORRUPT=1 run r04_rccl_corrupt 300 $TR --master-port 29622 bench.py --steps 10 --warmup 2 --no-walk-bench --no-cpu-baseline
rc=$?
if [ $rc -eq 0 ]; then echo "corrupted shard was NOT detected"; exit 1; fi
if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then echo "corrupt run timed out"; exit 1; fi
echo "corrupted shard detected (rc=$rc)"
run r04_tests_trainer 900 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_mt.py -x -q -p no:cacheprovider -rf --timeout 600 --timeout-method thread
