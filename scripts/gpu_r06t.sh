#!/bin/bash
# Round 6: the per-rank device footprint at C5 — rank 0 of an emulated
# W = 8 owner-layout job (lazy and sharded in-table exchange), the one-GPU C5 line, and the C5
# sub-line's walk / step peaks (hbm_peak_bytes* fields). Logs gpurun_out/r06t_*.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for x in lazy sharded; do
  timeout -k 10 400 python bench.py --config c5 --emulate-world 8 --in-exchange $x --steps 4 --warmup 1 \
    --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 > gpurun_out/r06t_w8_$x.log 2>&1 || { tail -10 gpurun_out/r06t_w8_$x.log; exit 1; }
  grep '^{' gpurun_out/r06t_w8_$x.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 emulated W=8 $x', round(d['ms_per_step'],2), d['hbm_peak_bytes'])"
done
timeout -k 10 400 python bench.py --config c5 --steps 4 --warmup 1 --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 > gpurun_out/r06t_n1.log 2>&1 || { tail -10 gpurun_out/r06t_n1.log; exit 1; }
grep '^{' gpurun_out/r06t_n1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 N=1', round(d['ms_per_step'],2), d['hbm_peak_bytes'])"
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 --batch64-steps 0 --c5-steps 4 > gpurun_out/r06t_c5sub.log 2>&1 || { tail -10 gpurun_out/r06t_c5sub.log; exit 1; }
grep '^{' gpurun_out/r06t_c5sub.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['c5']; print('c3 line', d['hbm_peak_bytes'], 'c5 walks', c['hbm_peak_bytes_walks'], 'c5 step', c['hbm_peak_bytes_step'], c['step_check']['ok'])"
