#!/bin/bash
# Round-6 evidence, part 1: the whole GPU suite, smoke() and the default bench line (with the
# C5 sub-line). Logs under gpurun_out/ (copied into profiles/ as r06_*).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/r06_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r06_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r06_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1 || { tail -10 gpurun_out/r06_smoke.log; exit 1; }
tail -1 gpurun_out/r06_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r06_bench.log 2>&1 || { tail -10 gpurun_out/r06_bench.log; exit 1; }
grep '^{' gpurun_out/r06_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['batch64']['ms_per_step'], d['c5']['ms_per_step'] if d.get('c5') else None)"
