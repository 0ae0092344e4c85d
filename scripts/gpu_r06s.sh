#!/bin/bash
# Round 6 A/B: k_out_rows' explicit vmcnt(0) at the row start (waits for the previous row's
# stores too) against none (the compiler's own waits at the loop latch cover the prefetched
# loads; libdw_hip_nowait.so), batch64 interleaved; the rows-major tests on the variant.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=deepwalk-and-node2vec_amd/shallow_encoders/_lib
DW_LIB_PATH=$PWD/$L/libdw_hip_nowait.so timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_gpu_owner.py tests/test_gpu_exact.py tests/test_gpu_graphed.py \
  tests/test_gpu_c3_step.py > gpurun_out/r06s_tests.log 2>&1 || { tail -40 gpurun_out/r06s_tests.log; exit 1; }
tail -1 gpurun_out/r06s_tests.log
for r in 1 2 3; do
  for v in wait nowait; do
    lib=$L/libdw_hip.so; [ $v = nowait ] && lib=$L/libdw_hip_nowait.so
    DW_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 > gpurun_out/r06s_${v}_$r.log 2>&1 || { tail -5 gpurun_out/r06s_${v}_$r.log; exit 1; }
    grep '^{' gpurun_out/r06s_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('$v', round(b['ms_per_step'],4), b['step_check']['ok'])"
  done
done
