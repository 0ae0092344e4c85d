#!/bin/bash
# Round 6: the N > 1 rows-major lazy path (two gloo ranks on one GPU, float and deterministic),
# the walkers' counted launches, then the bench line (walk rooflines with line moves, c5).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_owner.py -k "lazy" > gpurun_out/r06b_owner.log 2>&1 || { tail -40 gpurun_out/r06b_owner.log; exit 1; }
tail -3 gpurun_out/r06b_owner.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_walks.py > gpurun_out/r06b_walks.log 2>&1 || { tail -30 gpurun_out/r06b_walks.log; exit 1; }
tail -2 gpurun_out/r06b_walks.log
timeout -k 10 600 python -u bench.py > gpurun_out/r06b_bench.log 2>&1 || { tail -20 gpurun_out/r06b_bench.log; exit 1; }
grep '^{' gpurun_out/r06b_bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d.get('c5',{})
print('headline', d['value'], d['ms_per_step'], 'b64', d['batch64']['ms_per_step'])
for k in ('node2vec','node2vec_replay'): print(k, json.dumps(d['roofline_walk'].get(k,{}).get('random_line_roofline')))
for k in ('exact_walker','philox_walker'): print('c5', k, json.dumps(c.get(k,{}).get('roofline')))"
