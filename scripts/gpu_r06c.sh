#!/bin/bash
# Round 6: the pipelined / graphed lazy step with the counter ring (correctness), the N > 1
# rows-major tests, then the batch64 line under the capture-order variants, interleaved twice,
# and the headline under the in-table Adam grid scales.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_graphed.py "tests/test_gpu_exact.py::test_exact_lazy_rows_major_repeatable_and_equal_dense" \
  tests/test_gpu_owner.py -k "graphed or pipelined or lazy" > gpurun_out/r06c_tests.log 2>&1 || { tail -40 gpurun_out/r06c_tests.log; exit 1; }
tail -3 gpurun_out/r06c_tests.log
for i in 1 2; do
  for v in base centre early both; do
    ce=0; ie=0
    [ $v = centre ] && ce=1; [ $v = early ] && ie=1; [ $v = both ] && { ce=1; ie=1; }
    DW_PIPE_CENTRE_FIRST=$ce DW_PIPE_IN_EARLY=$ie timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 > gpurun_out/r06c_$v$i.log 2>&1 || { tail -5 gpurun_out/r06c_$v$i.log; exit 1; }
    grep '^{' gpurun_out/r06c_$v$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['batch64']; print('$v', b['ms_per_step'], b['roofline']['ms_per_step_events'], b['step_check']['ok'])"
  done
done
for i in 1 2; do
  for sc in 1.0 1.1 1.2 0.9; do
    DW_OVERLAP_SCALE=$sc timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 --batch64-steps 0 > gpurun_out/r06c_ov$sc$i.log 2>&1 || { tail -5 gpurun_out/r06c_ov$sc$i.log; exit 1; }
    grep '^{' gpurun_out/r06c_ov$sc$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('overlap $sc', d['ms_per_step'], r['in_table_adam_blocks'], r['ms_per_launch'])"
  done
done
