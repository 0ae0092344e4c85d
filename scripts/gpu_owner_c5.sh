#!/bin/bash
# Owner-computes emulations beyond the C3 sweep: rank 0's share of an 8-rank job on one GPU for
# C3 with the touched-row (lazy) in-table exchange and for C5 (R-MAT 24, d=256, node2vec
# p=.25 q=4) with both in-table exchanges. Stops at the first failure.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 3 "gpurun_out/$name.log"
  return $rc
}
step owner_emu_w8_lazy 300 python bench.py --emulate-world 8 --in-exchange lazy --steps 20 \
  --warmup 3 --no-cpu-baseline --no-walk-bench || exit 1
step owner_emu_c5_w8_lazy 600 python bench.py --config c5 --emulate-world 8 --in-exchange lazy \
  --steps 6 --warmup 2 --no-cpu-baseline --no-walk-bench || exit 1
step owner_emu_c5_w8_sharded 600 python bench.py --config c5 --emulate-world 8 \
  --in-exchange sharded --steps 6 --warmup 2 --no-cpu-baseline --no-walk-bench || exit 1
