#!/bin/bash
# Round 6: the new / changed GPU tests (range flag, first-step loss checks, Philox walker choice,
# C5 exact walker vs the oracle), then the default bench line (with its new c5 part).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_exact.py tests/test_gpu_c5_walks.py tests/test_gpu_bench.py \
  "tests/test_gpu_trainer.py::test_train_loop_replays_graphs_equal_to_eager" \
  "tests/test_gpu_trainer.py::test_reference_streams_c2_loop_graphed" \
  -k "not two_ranks" > gpurun_out/r06a_tests.log 2>&1 || { tail -30 gpurun_out/r06a_tests.log; exit 1; }
tail -3 gpurun_out/r06a_tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/r06a_bench.log 2>&1 || { tail -20 gpurun_out/r06a_bench.log; exit 1; }
grep '^{' gpurun_out/r06a_bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d.get('c5',{})
print('headline', d['value'], d['ms_per_step'], 'b64', d['batch64']['ms_per_step'])
print('c5', json.dumps({k: c.get(k) for k in ('walks_per_s_exact','walks_per_s_philox','ms_per_step','value','skipped')}))
print('c5 check', c.get('step_check'))
print('n2v roof', json.dumps(d['roofline_walk'].get('node2vec',{}).get('random_line_roofline')))
print('n2v replay roof', json.dumps(d['roofline_walk'].get('node2vec_replay',{}).get('random_line_roofline')))"
