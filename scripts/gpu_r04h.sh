#!/bin/bash
# Round 4: the box replay driven by the history header (row 0): the exhaustive /
# random bit checks against sqrtf and the IEEE division, the replay / owner / graphed / exact
# tests, C3 at 64 walks and its kernel trace, and the default bench line.
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
run r04h_box_check 120 ./scripts/microbench/box_check || exit 1
run r04h_replay_bench 120 ./scripts/microbench/replay_bench || exit 1
run r04h_tests 900 python -u -m pytest tests/test_gpu_owner.py tests/test_gpu_graphed.py tests/test_gpu_c3_step.py tests/test_gpu_exact.py -x -q -p no:cacheprovider -rf --timeout 600 --timeout-method thread || exit 1
for i in 1 2; do
  run r04h_c3_64_$i 300 python bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench --exact-steps 0 || exit 1
  grep '^{' gpurun_out/r04h_c3_64_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3/64', d['ms_per_step'])"
done
bash scripts/gpu_trace_c3_64.sh || exit 1
run r04h_bench_default 600 python bench.py || exit 1
