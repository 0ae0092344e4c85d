#!/bin/bash
# HBM bytes per kernel of the 64-walk C3 step (rocprofv3 --pmc, one counter per pass: FETCH_SIZE
# and WRITE_SIZE cannot share a pass on gfx950), the rows-major step and the catch-up / pass 1 /
# gather sequence (DW_OUT_ROWS=0: an A/B switch while round 4 measured it, since removed — a rerun
# now measures the default form twice). Output: gpurun_out/pmc64/<rows>_<counter>.csv
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmc64
export TMPDIR=/tmp
for rows in 1 0; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    DW_OUT_ROWS=$rows timeout -s KILL 300 rocprofv3 --pmc $ctr -d gpurun_out/pmc64/r${rows}_$ctr -o run --output-format csv -- python3 bench.py --batch-walks 64 --steps 16 --warmup 4 --no-cpu-baseline --no-walk-bench --exact-steps 0 > gpurun_out/pmc64/r${rows}_$ctr.log 2>&1 || { echo "pass $rows $ctr failed"; tail -5 gpurun_out/pmc64/r${rows}_$ctr.log; exit 1; }
    f=$(find gpurun_out/pmc64/r${rows}_$ctr -name "*counter_collection.csv" | head -1)
    cp "$f" gpurun_out/pmc64/r${rows}_$ctr.csv
    rm -rf gpurun_out/pmc64/r${rows}_$ctr
    echo "rows=$rows $ctr done"
  done
done
ls -la gpurun_out/pmc64
