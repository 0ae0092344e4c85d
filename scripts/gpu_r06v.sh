#!/bin/bash
# Round 6: kernel stats of the 64-walk step at steady state (20,000 graph-replayed steps after
# the headline) — which kernel grows with the in rows' lags. Outputs gpurun_out/r06v_*.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/r06v -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-walk-bench --exact-steps 0 --c5-steps 0 --batch64-steps 20000 > gpurun_out/r06v.log 2>&1 || { tail -5 gpurun_out/r06v.log; exit 1; }
f=$(find gpurun_out/r06v -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r06v_kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/r06v_kernel_stats.csv')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:12]:
    print(r['Name'][:70], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), round(float(r['MaxNs']) / 1e3, 1))
PY
f=$(find gpurun_out/r06v -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, statistics
ks = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in csv.DictReader(open(sys.argv[1])))
ca = [k for k in ks if 'k_rows_adam<false' in k[2]]
last = ca[-2000:]
print('in-row catch-up, last 2000 launches: median', statistics.median((e - s) / 1e3 for s, e, _ in last), 'us; max', max((e - s) / 1e3 for s, e, _ in last))
outs = [k for k in ks if 'k_out_rows' in k[2]][-2000:]
per = [(outs[i + 1][0] - outs[i][0]) / 1e3 for i in range(len(outs) - 1)]
print('period, last 2000 steps: median', statistics.median(per), 'us; k_out_rows median', statistics.median((e - s) / 1e3 for s, e, _ in outs))
PY
rm -rf gpurun_out/r06v
