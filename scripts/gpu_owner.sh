#!/bin/bash
# Owner-computes (N > 1 layout) session on a 1-GPU box: GPU tests of the owner kernels, then
# rank 0's share of W = 2/4/8 jobs emulated on the one GPU (no collectives), then a 2-rank
# rehearsal of the real multi-rank flow (gloo, both ranks on the device). Stops at the first
# failing GPU step.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  return $rc
}
step owner_tests 600 python -u -m pytest tests/test_gpu_owner.py -x -v -p no:cacheprovider \
  --timeout 300 --timeout-method thread || exit 1
for W in ${EMU_WORLDS:-2 4 8}; do
  step "owner_emu_w$W" 300 python bench.py --emulate-world "$W" --steps 20 --warmup 3 \
    --no-cpu-baseline --no-walk-bench ${BENCH_ARGS:-} || exit 1
done
step owner_rehearsal 300 env DW_BENCH_BACKEND=gloo DW_BENCH_ONE_DEVICE=1 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 4 --warmup 1 --no-cpu-baseline \
  --no-walk-bench || exit 1
