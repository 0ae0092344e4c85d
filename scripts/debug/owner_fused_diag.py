"""Debug: owner pass 2 with the fused slice Adam vs pass 2 + dw_adam_dense, per row and step."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, 'deepwalk-and-node2vec_amd'), REPO]
import numpy as np
import torch
from shallow_encoders.word2vec.sgns import sgns_owner_pass1, sgns_owner_pass2
from shallow_encoders.word2vec.sharding import adam_scalars, hip_adam, OwnerTables

V, D, R, K, L, NW, STEPS, LR = 700, 64, 2, 3, 12, 48, 3, 1e-3
g = torch.Generator().manual_seed(8)
walks = torch.randint(1, V, (STEPS, NW, L), generator=g, dtype=torch.int32)
per = L - 2 * R
W, r = 2, 1
tf = OwnerTables(V, D, 'cuda:0', lr=LR, init_seed=4, emulate_world=W)
S = tf.S
rows = torch.arange(S) * W + r
full_in = tf.w_in.clone()
gen = torch.Generator(device='cpu').manual_seed(4)
import math
a = math.sqrt(6.0 / (V + D))
w_in0 = torch.rand((V, D), generator=gen) * (2 * a) - a
w_out0 = torch.rand((V, D), generator=gen) * (2 * a) - a
w_in = w_in0.cuda()
fused = [w_out0[rows].cuda().contiguous()] + [torch.zeros((S, D), device='cuda') for _ in range(3)]
plain = [t.clone() for t in fused]
flags = torch.zeros(S, dtype=torch.uint8, device='cuda')
for s in range(STEPS):
    wk = walks[s].cuda()
    for tabs, fuse in ((fused, True), (plain, False)):
        w, gg, m, v = tabs
        g_in = torch.zeros_like(w_in)
        sgns_owner_pass1(w_in, w, g_in, K, walks=wk, context_radius=R, owner=r, n_owners=W,
                         vocab_size=V, seed=11, noise_offset=s * NW * per,
                         grad_scale=1.0 / (NW * per * 2 * R))
        spec = ({'m': m, 'v': v, 'flags': flags,
                 'scalars': adam_scalars(s + 1, LR, (0.9, 0.999), 1e-8, 0.0)} if fuse else None)
        n = sgns_owner_pass2(w_in, w, gg, K, walks=wk, context_radius=R, out_adam=spec)
        if not fuse:
            hip_adam(w.view(-1), gg.view(-1), m.view(-1), v.view(-1), s + 1, LR, (0.9, 0.999),
                     1e-8, 0.0, True)
    torch.cuda.synchronize()
    diff = (fused[0] - plain[0]).abs().max(1).values.cpu()
    bad = torch.nonzero(diff > 1e-6).flatten().tolist()
    print('step', s, 'records', n, 'rows differing', bad[:20], 'max', float(diff.max()),
          'flags max', int(flags.max()))

# records of the last pass-2 call (the plain table's, step 2): is the sorted buffer sorted?
from shallow_encoders.word2vec import sgns as _s
ws = _s._WORKSPACES[torch.device('cuda', 0)]
cap = NW * per * 2 * R * (1 + K)
kb = (cap * 4 + 255) // 256 * 256
vb = (cap * 8 + 255) // 256 * 256
k0 = ws[:cap * 4].view(torch.int32)[:n].cpu().numpy()
k1 = ws[kb:kb + cap * 4].view(torch.int32)[:n].cpu().numpy()
for name, k in (('k0', k0), ('k1', k1)):
    srt = bool(np.all(np.diff(k) >= 0))
    print(name, 'sorted', srt, 'min', k.min(), 'max', k.max(), 'count 348', int((k == 348).sum()),
          'positions of 348', np.nonzero(k == 348)[0][:12])
