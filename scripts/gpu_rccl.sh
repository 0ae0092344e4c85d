#!/bin/bash
# The N > 1 bench flow over RCCL on a one-GPU box: one rank in an 'nccl' process group with
# DW_BENCH_DIST=1 (collectives forced at world 1: calibration of both in-table exchanges, the
# replicated layout, strong scaling, node2vec's walk all-gather). A check of the RCCL calls, not
# a scaling measurement. Every GPU step has its own time limit; a failure stops the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp DW_BENCH_DIST=1
run() {  # run <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 4 "gpurun_out/$name.log"
  return $rc
}
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
run rccl_test 400 python -u -m pytest tests/test_gpu_rccl.py -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider || exit 1
run rccl_c3_auto 300 $TR --master-port 29611 bench.py --steps 20 --warmup 3 --no-walk-bench || exit 1
run rccl_c3_replicated 300 $TR --master-port 29612 bench.py --steps 20 --warmup 3 --no-walk-bench \
    --dist-mode replicated || exit 1
run rccl_c3_strong 300 $TR --master-port 29613 bench.py --steps 20 --warmup 3 --no-walk-bench \
    --scaling strong --in-exchange lazy || exit 1
run rccl_c2 300 $TR --master-port 29614 bench.py --config c2 --steps 40 --warmup 3 --no-walk-bench || exit 1
run rccl_c5 400 $TR --master-port 29615 bench.py --config c5 --steps 5 --warmup 2 --no-walk-bench || exit 1
