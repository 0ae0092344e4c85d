#!/bin/bash
# Round 6: batch64 A/B (interleaved): the next step's side chain captured before / after the out
# rows (DW_PIPE_FORK_LATE), the out rows' block ranges per resident slot (DW_OUT_ROWS_FACTOR 2 /
# 3 / 4), the graph captured and replayed on a high-priority stream (DW_GRAPH_HP).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 > gpurun_out/r06l_$name.log 2>&1 || { tail -5 gpurun_out/r06l_$name.log; exit 1; }
  grep '^{' gpurun_out/r06l_$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('$name', round(b['ms_per_step'], 4), b['step_check']['ok'])"
}
for i in 1 2; do
  run base$i DW_X=0
  run forklate$i DW_PIPE_FORK_LATE=1
  run fac3_$i DW_OUT_ROWS_FACTOR=3
  run fac4_$i DW_OUT_ROWS_FACTOR=4
  run hp$i DW_GRAPH_HP=1
done
