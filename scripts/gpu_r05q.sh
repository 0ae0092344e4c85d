#!/bin/bash
# Round 5: the pipelined 64-walk step's enqueue order (the side chains before or after the
# centre pass in the capture) — the graphed tests both ways, the 64-walk line both ways (twice).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
DW_PIPE_ORDER=main timeout -k 10 600 $T tests/test_gpu_graphed.py > gpurun_out/r05q_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05q_tests.log; [ $rc -eq 0 ] || exit $rc
for o in side main side main; do
  DW_PIPE_ORDER=$o timeout -k 10 300 python bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench > gpurun_out/r05q_$o.log 2>&1 || { tail -5 gpurun_out/r05q_$o.log; exit 1; }
  grep '^{' gpurun_out/r05q_$o.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$o', d['ms_per_step'], d['value'])"
done
