#!/bin/bash
# Round 4, first box: smoke, the GPU tests touched this round (walks, MT, owner / lazy / graphed,
# the full-size C3 step), then C3 at the reference's 64-walk batch and the default line.
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
  tail -n 25 "gpurun_out/$name.log"
  return $rc
}
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run r04_tests_a 900 python -u -m pytest tests/test_gpu_mt.py tests/test_gpu_walks.py tests/test_gpu_owner.py tests/test_gpu_graphed.py tests/test_gpu_c3_step.py -x -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: pytest rc=$rc"; exit $rc; fi
run r04_c3_64 300 python bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench || exit 1
run r04_bench 600 python bench.py --no-cpu-baseline --no-walk-bench || exit 1
