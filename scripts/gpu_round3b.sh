#!/bin/bash
# presort tests + C3/64 (gpu_presort.sh), node2vec replay rates for the counts kernel's
# occupancy variants, the training-loop reproducibility experiment. Logs under gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_presort.sh || exit 1
for v in default cn0; do
  if [ "$v" = cn0 ]; then export DW_N2V_CN_KERNEL=0; else unset DW_N2V_CN_KERNEL; fi
  timeout -k 10 300 python -u scripts/microbench/replay_rates.py --dw-walks 0 > gpurun_out/rates_$(basename $v).log 2>&1 || { tail -5 gpurun_out/rates_$(basename $v).log; exit 1; }
  echo "$v"; python3 -c "import json; d=json.loads(open('gpurun_out/rates_$(basename $v).log').read().strip().splitlines()[-1]); print({k:(round(x['kernel_ms'],2) if isinstance(x,dict) and 'kernel_ms' in x else x) for k,x in d.items()})"
done
unset DW_LIB_PATH
timeout -k 10 400 python -u scripts/experiments/train_graph_repro.py 2 > gpurun_out/train_repro.log 2>&1
grep -v "^[│├└ ]" gpurun_out/train_repro.log | grep -v "^\s" | tail -20
