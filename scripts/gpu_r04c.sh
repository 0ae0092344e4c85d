#!/bin/bash
# Round 4: the N > 1 bench flow over RCCL on one GPU (DW_BENCH_DIST=1, one 'nccl' rank) with its
# new self-check fields (rccl_world, exposed collective ms, step_check), the same with a
# corrupted shard (must exit non-zero), then the graphed-loop tests with the reference's streams.
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
  tail -n 4 "gpurun_out/$name.log" | cut -c1-600
  return $rc
}
# C3 at 64 walks: records per lazy-gather chunk (more waves in flight for the latency-bound gather)
for cfg in "64 1" "64 0" "32 1" "64 1"; do
  set -- $cfg
  DW_GCH=$1 DW_OUT_AHEAD=$2 run r04_c3_64_gch$1_ahead$2 300 python bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench --exact-steps 0 || exit 1
  grep '^{' gpurun_out/r04_c3_64_gch$1_ahead$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('gch $1 ahead $2', d['ms_per_step'])"
done
BENCH_ARGS="" bash scripts/gpu_trace_c3_64.sh || exit 1
run r04_owner_graphed_tests 900 python -u -m pytest tests/test_gpu_owner.py tests/test_gpu_graphed.py -x -q -p no:cacheprovider -rf --timeout 600 --timeout-method thread || exit 1
run r04_exact_loop 600 python -u -m pytest tests/test_gpu_exact.py -x -q -p no:cacheprovider -rf --timeout 500 --timeout-method thread -k train_loop
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
DW_BENCH_DIST=1 run r04_rccl_check 300 $TR --master-port 29621 bench.py --steps 20 --warmup 3 --no-walk-bench --no-cpu-baseline || exit 1
DW_BENCH_DIST=1 DW_BENCH_CORRUPT=1 run r04_rccl_corrupt 300 $TR --master-port 29622 bench.py --steps 10 --warmup 2 --no-walk-bench --no-cpu-baseline
rc=$?
if [ $rc -eq 0 ]; then echo "corrupted shard was NOT detected"; exit 1; fi
if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then echo "corrupt run timed out"; exit 1; fi
echo "corrupted shard detected (rc=$rc)"
run r04_tests_trainer 900 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_mt.py -x -q -p no:cacheprovider -rf --timeout 600 --timeout-method thread
