# Pass-2 chunk size sweep at C3 (DW_GCH: records per wave chunk; the product uses 512).
set -u
for c in 256 512 1024 2048; do
  DW_GCH=$c timeout -k 10 200 python bench.py --steps 200 --no-cpu-baseline --no-walk-bench > gpurun_out/gch_$c.log 2>&1 || exit 1
  echo "$c $(grep '^{' gpurun_out/gch_$c.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), round(d["roofline"]["phases"]["pass2"]["ms"],3))')"
done
