"""One node2vec replay launch at C3 (65,536 walks of L = 80, uniforms resident) — for rocprofv3
counter passes (scripts/gpu_pmc_replay.sh)."""
import os
import random
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, 'deepwalk-and-node2vec_amd'))

from shallow_encoders.graph.random_walk_generator import Node2Vec  # noqa: E402
from shallow_encoders.graph.rmat import rmat_graph  # noqa: E402
from shallow_encoders.graph.rng import draw_uniforms  # noqa: E402

dev = torch.device('cuda', 0)
csr = rmat_graph(20, 10_000_000, 0, device=dev)
L, n = 80, 65_536
layout = os.environ.get('DW_LAYOUT', 'indexed')
w = Node2Vec(csr, L, p=0.25, q=4.0, device=dev, layout=layout)
st = torch.arange(1, n + 1, dtype=torch.int32, device=dev)
u = torch.from_numpy(draw_uniforms(n * (L - 1), random.Random(0))).to(dev)
out = torch.empty((n, L), dtype=torch.int32, device=dev)
w.walk_batch(st[:64], uniforms=u[:64 * (L - 1)], out=out[:64])
w.walk_batch(st, uniforms=u, out=out)
torch.cuda.synchronize()
print('done', layout)
