#!/bin/bash
# C3 at 1,024 walks (4.3M records): the 11-bit 4K-tile sort (DW_SORT_SMALL11_MAX=8388608) vs the
# large-sort config (16K tiles), twice each.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in 4194304 8388608 4194304 8388608; do
  DW_SORT_SMALL11_MAX=$m timeout -k 10 300 python bench.py --batch-walks 1024 --steps 100 --no-cpu-baseline --no-walk-bench > gpurun_out/c3_1024_s11max_$m.log 2>&1 || { tail -5 gpurun_out/c3_1024_s11max_$m.log; exit 1; }
  grep '^{' gpurun_out/c3_1024_s11max_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('small11_max $m', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('phases'))"
done
