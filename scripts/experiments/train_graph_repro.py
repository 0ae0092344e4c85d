"""Reproducibility of tools/train.py's C2-shape loop: eager twice, graph-records, graph-auto;
epoch losses and table differences (is the eager loop itself run-to-run reproducible?).
DW_DETERMINISTIC=1 in the environment runs it in the deterministic accumulation mode."""
import os
import random
import sys
import tempfile

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, 'deepwalk-and-node2vec_amd'))
from tools import train as train_tool  # noqa: E402

base = ['datamodule.dataset_name=graph_rmat', 'datamodule.additional_parameters.scale=12',
        'datamodule.additional_parameters.n_edges=5429',
        'datamodule.additional_parameters.graph_seed=0',
        'datamodule.additional_parameters.walks_per_node=1',
        'datamodule.additional_parameters.method_params.q=1',
        'datamodule.additional_parameters.rng=philox', 'train.noise=device',
        'model.embedding_size=128', 'train.optimizer.lr=0.01',
        f'train.max_epochs={int(sys.argv[1]) if len(sys.argv) > 1 else 2}']
tmp = tempfile.mkdtemp()
res = {}
for tag, g, sc in (('eagerA', '0', 'auto'), ('eagerB', '0', 'auto'), ('graphR', '1', 'records'),
                   ('graphA', '1', 'auto')):
    os.environ['DW_TRAIN_GRAPH'] = g
    os.environ['DW_TRAIN_GRAPH_SCATTER'] = sc
    out = os.path.join(tmp, tag)
    torch.manual_seed(0)
    random.seed(0)   # the start-node shuffle draws from the global generator (datasets.py:45)
    last = train_tool.main(['--config-name', 'sge_sg_cora', f'path.output_dir={out}',
                            f'output_dir={out}', f'train.experiment={tag}'] + base)
    st = torch.load(os.path.join(out, 'graph_rmat', tag, 'checkpoints', 'last.ckpt'),
                    weights_only=True)
    res[tag] = (last, {k: v.numpy() for k, v in st['state_dict'].items()})
for tag in res:
    print(tag, {k: round(v, 6) for k, v in res[tag][0].items() if 'loss' in k}, flush=True)
for a, b in (('eagerA', 'eagerB'), ('eagerA', 'graphR'), ('eagerA', 'graphA')):
    for k in res[a][1]:
        x, y = res[a][1][k], res[b][1][k]
        d = np.abs(x - y)
        print(a, b, k, 'max', float(d.max()), 'frac>1e-6', float((d > 1e-6).mean()), flush=True)
