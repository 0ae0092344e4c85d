#!/bin/bash
# Multi-rank rehearsal on a 1-GPU box (gloo, all ranks on the device): the N > 1 bench flow in
# both scalings and both layouts, each step with its own time limit; stops at the first failure.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
port=29531
step() {  # step <name> <nproc> <bench args...>
  local name=$1 np=$2; shift 2
  port=$((port + 1))
  echo "=== $name ($(date +%T))"
  timeout -k 10 300 env DW_BENCH_BACKEND=gloo DW_BENCH_ONE_DEVICE=1 \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node "$np" --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus "$np" --steps 4 --warmup 1 --no-cpu-baseline \
    --no-walk-bench "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  grep '^{' "gpurun_out/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['scaling'], d['config']['global_batch_walks'], '%.3g pairs/s' % d['value'], d['in_exchange'], d['config']['parallelism'][:60])" || tail -n 25 "gpurun_out/$name.log"
  return $rc
}
step reh_weak 2 || exit 1
step reh_strong 2 --scaling strong || exit 1
step reh_replicated 2 --dist-mode replicated || exit 1
step reh_c2_w2 2 --config c2 || exit 1
