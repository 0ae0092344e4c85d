#!/bin/bash
# Quick tuning pass: SGNS parity tests, then bench variants (no CPU baseline / walk bench).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest ${TUNE_TESTS:-tests/test_gpu_sgns.py} -q -p no:cacheprovider -rf --timeout 300 > gpurun_out/tune_tests.log 2>&1
rc=$?; tail -3 gpurun_out/tune_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in ${TUNE_VARIANTS:-"DW_SGNS_G16=1" "DW_SGNS_G16=0"}; do
  echo "=== $v"
  env $v timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline ${TUNE_BENCH_FLAGS:---no-walk-bench} ${BENCH_ARGS:-} > gpurun_out/tune_bench.log 2>&1 || exit 1
  python -c "import json;r=json.loads(open('gpurun_out/tune_bench.log').read().splitlines()[-1]);print('value %.3g ms/step %.2f' % (r['value'], r['ms_per_step']), r['kernel_ms'], 'walks/s', r.get('walks_per_s'), r.get('walks_per_s_node2vec_p0.25_q4'))"
done
