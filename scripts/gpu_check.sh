#!/bin/bash
# One GPU-box session: smoke -> GPU parity tests -> short bench. Every GPU step has its own time
# limit; a fault/abort/timeout stops the script (no further GPU work in this call).
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
  tail -n 30 "gpurun_out/$name.log"
  return $rc
}
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run gpu_tests 1200 python -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 600
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: pytest rc=$rc"; exit $rc; fi
run bench 900 python bench.py ${BENCH_ARGS:-} || exit 1
