#!/bin/bash
# Round 6 A/B: k_out_rows at 6 / 7 / 8 (and 5) waves per SIMD (OUT_ROWS_WAVES; 7 and 8 spill),
# batch64 interleaved twice. Variant libraries via DW_LIB_PATH (timing only).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=deepwalk-and-node2vec_amd/shallow_encoders/_lib
for r in 1 2 3; do
  for v in 6 7 8; do
    lib=$L/libdw_hip.so; [ $v != 6 ] && lib=$L/libdw_hip_w$v.so
    DW_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 > gpurun_out/r06o_${v}_$r.log 2>&1 || { tail -5 gpurun_out/r06o_${v}_$r.log; exit 1; }
    grep '^{' gpurun_out/r06o_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('waves $v', round(b['ms_per_step'],4), b['step_check']['ok'])"
  done
done
