#!/bin/bash
# Round 6 A/B: the centre pass (COEFIN k_sgns_g16) with the next chunk's rows in flight
# (DW_COEFIN_PIPE 1, the built library) against the plain chunk loop (libdw_hip_nopipe.so).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=deepwalk-and-node2vec_amd/shallow_encoders/_lib
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_gpu_owner.py tests/test_gpu_exact.py tests/test_gpu_graphed.py \
  tests/test_gpu_c3_step.py > gpurun_out/r06r_tests.log 2>&1 || { tail -40 gpurun_out/r06r_tests.log; exit 1; }
tail -1 gpurun_out/r06r_tests.log
for r in 1 2 3; do
  for v in pipe nopipe; do
    lib=$L/libdw_hip.so; [ $v = nopipe ] && lib=$L/libdw_hip_nopipe.so
    DW_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 > gpurun_out/r06r_${v}_$r.log 2>&1 || { tail -5 gpurun_out/r06r_${v}_$r.log; exit 1; }
    grep '^{' gpurun_out/r06r_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('$v', round(b['ms_per_step'],4), b['step_check']['ok'], round(d['ms_per_step'],3))"
  done
done
bash scripts/gpu_prof_c3_64.sh > gpurun_out/r06r_prof.log 2>&1 || { tail -5 gpurun_out/r06r_prof.log; exit 1; }
