#!/bin/bash
# tools/train.py's loop with graph-replayed steps: the trainer / graph tests, then the C2 shape
# (Cora-sized R-MAT, node2vec p=1 q=1, L=10, R=2, 64-walk batches, d=128, 16 walks per node:
# 1,024 steps per epoch) timed with the graphs on and off; the small-sort configs.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/microbench/small_sort_bench > gpurun_out/small_sort_bench.log 2>&1 || { tail -3 gpurun_out/small_sort_bench.log; exit 1; }
cat gpurun_out/small_sort_bench.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_graphed.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/train_graph_tests.log 2>&1; rc=$?
tail -3 gpurun_out/train_graph_tests.log
[ $rc -eq 0 ] || exit $rc
cd deepwalk-and-node2vec_amd
for g in 0 1; do
  DW_TRAIN_GRAPH=$g timeout -k 10 300 python tools/train.py --config-name=sge_sg_cora path.output_dir=/tmp/c2run$g output_dir=/tmp/c2run$g \
    datamodule.dataset_name=graph_rmat datamodule.additional_parameters.scale=12 datamodule.additional_parameters.n_edges=5429 \
    datamodule.additional_parameters.method_params.q=1 datamodule.additional_parameters.rng=philox train.noise=device \
    model.embedding_size=128 train.max_epochs=3 > ../gpurun_out/train_c2_graph$g.log 2>&1 || { tail -5 ../gpurun_out/train_c2_graph$g.log; exit 1; }
  echo "DW_TRAIN_GRAPH=$g"; grep "^epoch" ../gpurun_out/train_c2_graph$g.log
done
