set -u
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --no-walk-bench > gpurun_out/pf_on.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --no-walk-bench --walk-prefetch > gpurun_out/pf_off.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --no-walk-bench > gpurun_out/pf_on2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --emulate-world 8 --steps 20 --no-cpu-baseline --no-walk-bench > gpurun_out/pf_w8.log 2>&1 || exit 1
timeout -k 10 300 env DW_BENCH_BACKEND=gloo DW_BENCH_ONE_DEVICE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --steps 4 --warmup 1 --no-cpu-baseline --no-walk-bench > gpurun_out/pf_reh.log 2>&1 || exit 1
timeout -k 10 300 env DW_BENCH_BACKEND=gloo DW_BENCH_ONE_DEVICE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --steps 4 --warmup 1 --no-cpu-baseline --no-walk-bench --dist-mode replicated > gpurun_out/pf_reh_rep.log 2>&1 || exit 1
