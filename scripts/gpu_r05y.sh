#!/bin/bash
# Round 5: HBM traffic of the 64-walk step on the final code — FETCH_SIZE and WRITE_SIZE passes
# over bench.py --batch-walks 64, summarised into profiles/sgns_pmc.json (c3_batch64) by
# scripts/pmc_batch64.py. Outputs gpurun_out/r05y_*.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --batch-walks 64 --steps 16 --warmup 4 --no-cpu-baseline --no-walk-bench --exact-steps 0 --batch64-steps 0"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/r05y_$c -o run --output-format csv -- $B > gpurun_out/r05y_$c.log 2>&1 || { echo "$c failed"; tail -3 gpurun_out/r05y_$c.log; exit 1; }
  f=$(find gpurun_out/r05y_$c -name "*counter_collection.csv" | head -1); cp "$f" gpurun_out/r05y_$c.csv; rm -rf gpurun_out/r05y_$c
done
mkdir -p gpurun_out/profiles
python3 scripts/pmc_batch64.py gpurun_out/r05y_FETCH_SIZE.csv gpurun_out/r05y_WRITE_SIZE.csv 20 r05 "bench.py --batch-walks 64 (lazy owner path, rows-major out step with block-shared rows, pipelined graph replay), 16 timed + 4 warmup steps; per launch 2*FETCH_SIZE + WRITE_SIZE (KiB->B) as in r01; hbm_bytes_per_step sums the per-step kernels (the bench line's algorithmic figure: 1030 MB/step)" && cp profiles/sgns_pmc.json gpurun_out/profiles/sgns_pmc.json
