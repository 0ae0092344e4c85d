#!/bin/bash
# Round-3 evidence, part 2: the small-sort configs, the other batch shapes (C3 at 64 and 1,024
# walks, the C2 shape), C5 on one GPU, tools/train.py on the C2 shape with graphs on / off.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/microbench/small_sort_bench > gpurun_out/small_sort_bench.log 2>&1 || { tail -3 gpurun_out/small_sort_bench.log; exit 1; }
cat gpurun_out/small_sort_bench.log
BATCH_SPECS="c3_64:--batch-walks 64 --steps 400;c3_1024:--batch-walks 1024 --steps 100;c2:--config c2 --steps 400" bash scripts/gpu_batches.sh || exit 1
timeout -k 10 400 python bench.py --config c5 --steps 30 --warmup 3 --no-cpu-baseline --no-walk-bench > gpurun_out/bench_c5.log 2>&1 || { tail -5 gpurun_out/bench_c5.log; exit 1; }
grep '^{' gpurun_out/bench_c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', d['value'], d['ms_per_step'], d['roofline']['frac'], {k: round(v['ms'],2) for k, v in d['roofline'].get('phases', {}).items()})"
cd deepwalk-and-node2vec_amd
for g in 1 0; do
  DW_TRAIN_GRAPH=$g timeout -k 10 300 python tools/train.py --config-name=sge_sg_cora path.output_dir=/tmp/c2run$g output_dir=/tmp/c2run$g \
    datamodule.dataset_name=graph_rmat datamodule.additional_parameters.scale=12 datamodule.additional_parameters.n_edges=5429 \
    datamodule.additional_parameters.method_params.q=1 datamodule.additional_parameters.rng=philox train.noise=device \
    model.embedding_size=128 train.max_epochs=3 > ../gpurun_out/train_c2_graph$g.log 2>&1 || { tail -5 ../gpurun_out/train_c2_graph$g.log; exit 1; }
  echo "DW_TRAIN_GRAPH=$g"; grep "^epoch" ../gpurun_out/train_c2_graph$g.log
done
