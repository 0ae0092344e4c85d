#!/bin/bash
# SQ counter passes over one node2vec replay launch (scripts/microbench/replay_once.py).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" ; do
  i=$((i+1))
  echo "=== pass $i: $grp"
  timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/pmc_replay_$i -o run --output-format csv -- \
    python3 scripts/microbench/replay_once.py > gpurun_out/pmc_replay_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_replay_$i.log; exit 1; }
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/replay_trace -o run --output-format csv -- python3 scripts/microbench/replay_once.py > gpurun_out/replay_trace.log 2>&1
