set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/microbench/partition_bench > gpurun_out/partition_bench.log 2>&1; rc=$?
cat gpurun_out/partition_bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_sgns.py -k "stream_copy" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -3
