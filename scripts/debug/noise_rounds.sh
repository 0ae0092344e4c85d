# Timing study: owner pass 1 at W=8 with the noise Philox at 10 rounds (product) vs 20 rounds
# (experimental build: the same law, twice the work) — how much of pass 1 the negative draws cost.
set -u
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python bench.py --emulate-world 8 --steps 20 --no-cpu-baseline --no-walk-bench > gpurun_out/nr_10.log 2>&1 || exit 1
DW_LIB_PATH=$PWD/scripts/debug/exp/libdw_hip_r20.so timeout -k 10 300 python bench.py --emulate-world 8 --steps 20 --no-cpu-baseline --no-walk-bench > gpurun_out/nr_20.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-walk-bench > gpurun_out/nr_10_n1.log 2>&1 || exit 1
DW_LIB_PATH=$PWD/scripts/debug/exp/libdw_hip_r20.so timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-walk-bench > gpurun_out/nr_20_n1.log 2>&1 || exit 1
