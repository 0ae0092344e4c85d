#!/bin/bash
# Round 6: the one-side-stream pipelined step — its parity tests, then the order of the two
# chains on the side stream (in-row chain first vs placement first), interleaved twice.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_gpu_graphed.py "tests/test_gpu_exact.py::test_exact_lazy_rows_major_repeatable_and_equal_dense" \
  "tests/test_gpu_c3_step.py" > gpurun_out/r06i_tests.log 2>&1 || { tail -40 gpurun_out/r06i_tests.log; exit 1; }
tail -1 gpurun_out/r06i_tests.log
for i in 1 2; do
  for v in 0 1; do
    DW_PIPE_OUT_FIRST=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 > gpurun_out/r06i_$v$i.log 2>&1 || { tail -5 gpurun_out/r06i_$v$i.log; exit 1; }
    grep '^{' gpurun_out/r06i_$v$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('out_first=$v', b['ms_per_step'], b['step_check']['ok'])"
  done
done
bash scripts/gpu_prof_c3_64.sh > gpurun_out/r06i_prof.log 2>&1 || { tail -5 gpurun_out/r06i_prof.log; exit 1; }
head -1 gpurun_out/r06i_prof.log
