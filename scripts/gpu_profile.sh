#!/bin/bash
# rocprofv3 passes over a short bench run (1 GPU): kernel trace + stats, then one PMC pass per
# counter group (never combined with tracing domains). Outputs under gpurun_out/prof_*.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--steps ${PROF_STEPS:-10} --warmup 2 --no-cpu-baseline --no-walk-bench ${BENCH_ARGS:-}"
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  return $rc
}
step prof_trace 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run \
  --output-format csv -- python3 bench.py $ARGS || exit 1
for ctr in FETCH_SIZE WRITE_SIZE TCC_EA0_ATOMIC_sum; do
  step "prof_pmc_$ctr" 600 rocprofv3 --pmc $ctr -d "gpurun_out/prof_pmc_$ctr" -o run \
    --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline \
    --no-walk-bench ${BENCH_ARGS:-} || exit 1
done
