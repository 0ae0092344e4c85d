"""Debug (round 6): two gloo ranks on one GPU, the lazy rows-major step, per-step flushed state
against one process, and per-step gradient G of the in rows."""
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, 'deepwalk-and-node2vec_amd'), REPO, os.path.join(REPO, 'tests')]
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

V, D, R, K, L, NW, STEPS, LR = 700, 64, 2, 3, 12, 48, 3, 1e-3


def run(rows_major: bool, exact: bool = False):
    from shallow_encoders.word2vec.sharding import OwnerLazyTables, owner_lazy_step
    t = OwnerLazyTables(V, D, 'cuda:0', lr=LR, init_seed=4, lazy_out=True)
    t.rows_major = rows_major
    per = L - 2 * R
    if exact:
        t.enable_exact(1.0 / (NW * per * 2 * R))
    g = torch.Generator().manual_seed(8)
    walks = torch.randint(1, V, (STEPS, NW, L), generator=g, dtype=torch.int32)
    acc = torch.zeros(4, dtype=torch.float64, device='cuda:0')
    st = torch.zeros(1, dtype=torch.int32, device='cuda:0')
    snaps = []
    for s in range(STEPS):
        owner_lazy_step(t, walks[s].cuda(), R, K, seed=11, noise_offset=s * NW * per,
                        grad_scale=1.0 / (NW * per * 2 * R), loss_acc=acc, status=st)
        torch.cuda.synchronize()
        G = t._G[:int(t._n_host[0])].cpu().clone() if t.multi else None
        U = t._touched[:int(t._n_touched.item())].cpu().clone()
        t.flush()
        snaps.append(([x[:V].cpu().clone() for x in (t.params_in[0], t.m_in, t.v_in)]
                      + [t.full_w_out().cpu()], G, U))
    return snaps


def worker(rank, q, exact):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = '29534'
    dist.init_process_group('gloo', rank=rank, world_size=2)
    try:
        out = run(True, exact)
        q.put((rank, [([x.numpy() for x in xs], None if G is None else G.numpy(), U.numpy())
                      for xs, G, U in out]))
    except Exception as e:
        import traceback
        q.put((rank, traceback.format_exc()))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == '__main__':
    for exact in (False, True):
        ref = run(True, exact)
        ctx = mp.get_context('spawn')
        q = ctx.Queue()
        ps = [ctx.Process(target=worker, args=(r, q, exact)) for r in range(2)]
        for p in ps:
            p.start()
        res = dict(q.get(timeout=300) for _ in range(2))
        for p in ps:
            p.join()
        if isinstance(res[0], str):
            print(res[0])
            continue
        print('exact', exact)
        for s in range(STEPS):
            x, G, U = res[0][s]
            y, _, U1 = ref[s]
            import numpy as np
            y = [t.numpy() for t in y]
            print('  step', s, ' '.join(f'{n}:{float(np.abs(p - q).max()):.2e}'
                                       for n, p, q in zip(('w_in', 'm_in', 'v_in', 'w_out'), x, y)),
                  '|U|', U.size, U1.numel())
            bad = np.nonzero((np.abs(x[1] - y[1]) > 1e-9).any(1))[0]
            print('    bad in rows', bad.size, bad[:10].tolist(), 'in U?', np.isin(bad[:10], U).tolist())
