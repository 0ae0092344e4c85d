#!/bin/bash
# Bench lines at other batch shapes (one GPU): the reference's 64-walk batch and 1,024 walks on
# C3, the W=8 global batch (65,536 walks) on one GPU, the C2 shape (default: the atomic
# scatter at this size) and with the records (sorted) scatter. Each run has its own time
# limit; a failure stops the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/batches.jsonl
: > $OUT
run() {  # run <name> <args...>
  local name=$1; shift
  echo "=== $name: $*"
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-walk-bench "$@" > gpurun_out/b_$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/b_$name.log; echo "rc=$rc"; exit $rc; fi
  grep '^{' gpurun_out/b_$name.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['run']='$name'; print(json.dumps(d))" >> $OUT
  python -c "import json; d=json.loads(open('$OUT').read().splitlines()[-1]); print(d['run'], '%.4g pairs/s' % d['value'], '%.3f ms/step' % d['ms_per_step'], 'frac %.3f' % d['roofline']['frac'])"
}
SPECS=${BATCH_SPECS:-"c3_64:--batch-walks 64 --steps 200;c3_1024:--batch-walks 1024 --steps 100;c3_65536:--batch-walks 65536 --steps 5;c2:--config c2 --steps 400;c2_sorted:--config c2 --scatter sorted --steps 400"}
IFS=';' read -ra ITEMS <<< "$SPECS"
for spec in "${ITEMS[@]}"; do
  name=${spec%%:*}; args=${spec#*:}
  IFS=' ' read -ra ARGV <<< "$args"
  run $name "${ARGV[@]}"
done
