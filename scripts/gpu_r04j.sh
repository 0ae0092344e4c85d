#!/bin/bash
# Round 4: rows-major step with the claim's slot rows (no second Philox draw), no counter memset,
# and the first round's centre rows loaded with the row — its tests, C3 at 64 walks, the trace.
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
  tail -n 3 "gpurun_out/$name.log" | cut -c1-300
  return $rc
}
run r04j_tests 900 python -u -m pytest tests/test_gpu_owner.py tests/test_gpu_graphed.py tests/test_gpu_c3_step.py -x -q -p no:cacheprovider -rf --timeout 600 --timeout-method thread || exit 1
for i in 1 2; do
  run r04j_c3_64_$i 300 python bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench --exact-steps 0 || exit 1
  grep '^{' gpurun_out/r04j_c3_64_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3/64', d['ms_per_step'])"
done
bash scripts/gpu_trace_c3_64.sh || exit 1
python3 scripts/trace_summary.py gpurun_out/trace64_kernel_trace.csv timeline | tail -14
