#!/bin/bash
# Round 4: C3 at 64 walks, lazy gather with the next row prefetched vs not (DW_LAZY_PREFETCH),
# its kernel trace, the owner / graphed tests, and tools/train.py on the
# C2 shape with the reference's own streams (rng python, noise torch) graphed vs eager.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 3 "gpurun_out/$name.log" | cut -c1-400
  return $rc
}
for g in 1 0 1; do
  DW_LAZY_PREFETCH=$g run r04f_c3_64_pf$g 300 python bench.py --batch-walks 64 --steps 400 --no-cpu-baseline --no-walk-bench --exact-steps 0 || exit 1
  grep '^{' gpurun_out/r04f_c3_64_pf$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('prefetch $g', d['ms_per_step'])"
done
bash scripts/gpu_trace_c3_64.sh || exit 1
run r04f_owner_graphed_tests 900 python -u -m pytest tests/test_gpu_owner.py tests/test_gpu_graphed.py tests/test_gpu_c3_step.py -x -q -p no:cacheprovider -rf --timeout 600 --timeout-method thread || exit 1
cd deepwalk-and-node2vec_amd
C2="datamodule.dataset_name=graph_rmat datamodule.additional_parameters.scale=12 datamodule.additional_parameters.n_edges=5429 datamodule.additional_parameters.method_params.q=1 model.embedding_size=128 train.max_epochs=3"
for cfg in "1 python torch" "0 python torch" "1 philox device"; do
  set -- $cfg
  DW_TRAIN_GRAPH=$1 timeout -k 10 300 python tools/train.py --config-name=sge_sg_cora path.output_dir=/tmp/c2r$1$2 output_dir=/tmp/c2r$1$2 \
    $C2 datamodule.additional_parameters.rng=$2 train.noise=$3 > ../gpurun_out/r04f_train_c2_g$1_$2.log 2>&1 || { tail -5 ../gpurun_out/r04f_train_c2_g$1_$2.log; exit 1; }
  echo "graph=$1 rng=$2 noise=$3"; grep "^epoch" ../gpurun_out/r04f_train_c2_g$1_$2.log
done
