#!/bin/bash
# PMC passes over the replay microbenchmark (one rocprofv3 --pmc run per counter group).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmc_replay
export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
            "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_WAVES" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs -d gpurun_out/pmc_replay/p$i -o run --output-format csv -- ./scripts/microbench/replay_bench 224000 3 > gpurun_out/pmc_replay/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_replay/p$i.log; exit 1; }
  f=$(find gpurun_out/pmc_replay/p$i -name "*counter_collection.csv" | head -1)
  cp "$f" gpurun_out/pmc_replay/pass$i.csv
  rm -rf gpurun_out/pmc_replay/p$i
done
ls -la gpurun_out/pmc_replay
