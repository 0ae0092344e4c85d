#!/bin/bash
# node2vec replay with per-edge class counts: the walk tests, then the C3 replay rates (with and
# without the counts) and a b_factor sweep. Logs under gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_walks.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/n2v_cn_tests.log 2>&1; rc=$?
tail -5 gpurun_out/n2v_cn_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/microbench/replay_rates.py --dw-walks 0 > gpurun_out/n2v_cn_rates.log 2>&1 || { tail -5 gpurun_out/n2v_cn_rates.log; exit 1; }
cat gpurun_out/n2v_cn_rates.log
for f in 4 64 256; do
  DW_N2V_BFACTOR=$f timeout -k 10 300 python -u scripts/microbench/replay_rates.py --dw-walks 0 > gpurun_out/n2v_cn_rates_f$f.log 2>&1 || { tail -5 gpurun_out/n2v_cn_rates_f$f.log; exit 1; }
  echo "F=$f"; cat gpurun_out/n2v_cn_rates_f$f.log
done
