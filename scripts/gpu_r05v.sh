#!/bin/bash
# Round 5: A/B of two builds of libdw_hip on one box (DW_LIB_PATH: the experimental build) — the
# 64-walk step (bench batch64 line), interleaved three times. Usage: gpu_r05v.sh <exp .so> <tag>
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
EXP=$1; TAG=$2
for i in 1 2 3; do
  for v in base exp; do
    if [ $v = exp ]; then export DW_LIB_PATH=$PWD/$EXP; else unset DW_LIB_PATH; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 > gpurun_out/r05v_${TAG}_$v$i.log 2>&1 || { tail -5 gpurun_out/r05v_${TAG}_$v$i.log; exit 1; }
    grep '^{' gpurun_out/r05v_${TAG}_$v$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('$TAG $v', b['ms_per_step'], b['value'], b['step_check']['ok'])"
  done
done
unset DW_LIB_PATH
