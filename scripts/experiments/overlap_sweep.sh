set -u
for b in 32 40 47 56 64 80; do
  DW_OVERLAP_BLOCKS=$b timeout -k 10 200 python bench.py --steps 200 --no-cpu-baseline --no-walk-bench > gpurun_out/sw_$b.log 2>&1 || exit 1
  echo "$b $(grep '^{' gpurun_out/sw_$b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), d["roofline"]["in_table_adam_blocks"])')"
done
