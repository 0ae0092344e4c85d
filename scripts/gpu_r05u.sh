#!/bin/bash
# Round 5: k_out_rows with chunk tickets (waves that finish early take more chunks) — the tests
# that run it, then the 64-walk step (bench batch64 line) at chunk sizes auto / 32 / 16.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_graphed.py tests/test_gpu_exact.py tests/test_gpu_owner.py > gpurun_out/r05u_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05u_tests.log; [ $rc -eq 0 ] || exit $rc
for g in auto 32 16 auto 32 16; do
  if [ $g = auto ]; then unset DW_OUT_ROWS_GCH; else export DW_OUT_ROWS_GCH=$g; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 > gpurun_out/r05u_bench_$g.log 2>&1 || { tail -5 gpurun_out/r05u_bench_$g.log; exit 1; }
  grep '^{' gpurun_out/r05u_bench_$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('gch $g batch64', b['ms_per_step'], b['value'], b['roofline']['frac'], b['step_check']['ok'])"
done
unset DW_OUT_ROWS_GCH
