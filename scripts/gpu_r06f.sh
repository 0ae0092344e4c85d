#!/bin/bash
# Round 6: the reference's 64-walk batch on the N > 1 path — the one-rank RCCL
# rehearsal (DW_BENCH_DIST=1: the whole N > 1 flow, collectives over a one-rank nccl group) with
# its step check, and rank 0 of an emulated W = 8 job (no collectives) for the projection.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
DW_BENCH_DIST=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29561 bench.py --batch-walks 64 --steps 200 --warmup 10 \
  --no-walk-bench > gpurun_out/r06f_rccl64.log 2>&1 || { tail -20 gpurun_out/r06f_rccl64.log; exit 1; }
grep '^{' gpurun_out/r06f_rccl64.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rccl world1 b64', d['ms_per_step'], d['in_exchange'], d['in_exchange_calibration_ms_per_step'], d['layout_calibration_ms_per_step'], d['step_check']['ok'], d['config']['parallelism'])"
for W in 1 2 4 8; do
  timeout -k 10 300 python bench.py --batch-walks 64 --emulate-world $W --in-exchange lazy --steps 200 --warmup 10 \
    --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 --batch64-steps 0 > gpurun_out/r06f_emu$W.log 2>&1 || { tail -10 gpurun_out/r06f_emu$W.log; exit 1; }
  grep '^{' gpurun_out/r06f_emu$W.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('emulated W=$W b64', d['ms_per_step'], d['value'], d['records_per_step_per_gpu'])"
done
