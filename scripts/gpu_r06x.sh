#!/bin/bash
# Round 6 A/B at the 64-walk step's steady state: k_out_rows at 7 / 6 / 5 waves per SIMD (the
# in rows' catch-up beside it gets the SIMDs' remaining wave slots), batch64 400 steps and the
# last 4,000 of 20,000. Variant libraries via DW_LIB_PATH (timing only).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=deepwalk-and-node2vec_amd/shallow_encoders/_lib
for r in 1 2; do
  for v in 7 6 5; do
    lib=$L/libdw_hip.so; [ $v != 7 ] && lib=$L/libdw_hip_w$v.so
    DW_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 > gpurun_out/r06x_${v}_$r.log 2>&1 || { tail -5 gpurun_out/r06x_${v}_$r.log; exit 1; }
    grep '^{' gpurun_out/r06x_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('waves $v', round(b['ms_per_step'],4), round(b['steady_state']['ms_per_step'],4), b['step_check']['ok'])"
  done
done
