#!/bin/bash
# Round 4: the rows-major lazy out step (dw_sgns_owner_out_rows + the coefficients-in centre
# pass) — its tests against the gather path and dense training, C3 at 64 walks rows-major vs
# the catch-up / pass 1 / gather path (DW_OUT_ROWS=0, an A/B switch since removed), and the kernel trace.
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
run r04i_rows_tests 600 python -u -m pytest tests/test_gpu_owner.py -x -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread -k "rows_major or lazy_single_rank or placed_records" || exit 1
run r04i_tests 900 python -u -m pytest tests/test_gpu_owner.py tests/test_gpu_graphed.py tests/test_gpu_c3_step.py tests/test_gpu_exact.py -x -q -p no:cacheprovider -rf --timeout 600 --timeout-method thread || exit 1
for cfg in "1 a" "0 b" "1 c"; do
  set -- $cfg
  DW_OUT_ROWS=$1 run r04i_c3_64_rows$1$2 300 python bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench --exact-steps 0 || exit 1
  grep '^{' gpurun_out/r04i_c3_64_rows$1$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rows-major $1', d['ms_per_step'])"
done
bash scripts/gpu_trace_c3_64.sh || exit 1
