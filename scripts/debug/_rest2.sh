set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/rest2_gpu_tests.log 2>&1 || { tail -30 gpurun_out/rest2_gpu_tests.log; exit 1; }
tail -1 gpurun_out/rest2_gpu_tests.log
rm -rf gpurun_out/rest2_prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/rest2_prof -o run --output-format csv -- python3 bench.py --config c5 --steps 6 --warmup 2 --no-cpu-baseline --no-walk-bench > gpurun_out/rest2_prof.log 2>&1 || { tail -20 gpurun_out/rest2_prof.log; exit 1; }
grep '^{' gpurun_out/rest2_prof.log | cut -c1-260
grep -h "k_adam_rest" gpurun_out/rest2_prof/run_kernel_stats.csv | rev | cut -d, -f1-6 | rev
