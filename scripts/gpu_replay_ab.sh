#!/bin/bash
# node2vec replay walker: rates of the in-tree build against variant builds
# (scripts/microbench/var/libdw_*.so), then the walk tests on the in-tree build.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/replay_ab.jsonl
for lib in default scripts/microbench/var/libdw_old.so scripts/microbench/var/libdw_pre1.so scripts/microbench/var/libdw_rbb16.so; do
  if [ "$lib" = default ]; then
    timeout -k 10 300 python scripts/microbench/replay_rates.py --dw-walks 0 >> gpurun_out/replay_ab.jsonl 2> gpurun_out/replay_ab.err || { tail -5 gpurun_out/replay_ab.err; exit 1; }
  else
    DW_LIB_PATH=$lib timeout -k 10 300 python scripts/microbench/replay_rates.py --dw-walks 0 >> gpurun_out/replay_ab.jsonl 2> gpurun_out/replay_ab.err || { tail -5 gpurun_out/replay_ab.err; exit 1; }
  fi
  tail -1 gpurun_out/replay_ab.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['lib'], {k: round(v['walks_per_s']) for k, v in d.items() if isinstance(v, dict) and 'walks_per_s' in v})"
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_walks.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/replay_walk_tests.log 2>&1; rc=$?
tail -3 gpurun_out/replay_walk_tests.log
exit $rc
