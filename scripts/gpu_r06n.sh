#!/bin/bash
# Round 6: counters of the 64-walk step (bench.py --batch-walks 64): SQ instruction / wait passes
# (k_out_rows' VALU issue per row) and the FETCH_SIZE / WRITE_SIZE passes that
# scripts/pmc_batch64.py summarises into profiles/sgns_pmc.json. Outputs gpurun_out/r06n_*.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --batch-walks 64 --steps 16 --warmup 4 --no-cpu-baseline --no-walk-bench --exact-steps 0 --batch64-steps 0 --c5-steps 0"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
           FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/r06n_$i -o run --output-format csv -- $B > gpurun_out/r06n_$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/r06n_$i.log; exit 1; }
  f=$(find gpurun_out/r06n_$i -name "*counter_collection.csv" | head -1); cp "$f" gpurun_out/r06n_$i.csv; rm -rf gpurun_out/r06n_$i
done
mkdir -p gpurun_out/profiles
python3 scripts/pmc_batch64.py gpurun_out/r06n_3.csv gpurun_out/r06n_4.csv 20 r06 "bench.py --batch-walks 64 (lazy owner path, rows-major out step with whole rows per range, pipelined graph replay), 16 timed + 4 warmup steps; per launch 2*FETCH_SIZE + WRITE_SIZE (KiB->B) as in r01; hbm_bytes_per_step sums the per-step kernels" && cp profiles/sgns_pmc.json gpurun_out/profiles/sgns_pmc.json
