"""Debug (round 6): the lazy rows-major step over a forced one-rank collective group
(DW_FORCE_COLLECTIVES=1, gloo) against the plain one-rank step, per step, flushed states."""
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, 'deepwalk-and-node2vec_amd'), REPO, os.path.join(REPO, 'tests')]
import torch
import torch.distributed as dist

V, D, R, K, L, NW, STEPS, LR = 700, 64, 2, 3, 12, 48, 3, 1e-3


def run(multi: bool, rows_major: bool):
    from shallow_encoders.word2vec.sharding import OwnerLazyTables, owner_lazy_step
    os.environ['DW_FORCE_COLLECTIVES'] = '1' if multi else '0'
    t = OwnerLazyTables(V, D, 'cuda:0', lr=LR, init_seed=4, lazy_out=True)
    t.rows_major = rows_major
    assert t.multi == multi
    g = torch.Generator().manual_seed(8)
    walks = torch.randint(1, V, (STEPS, NW, L), generator=g, dtype=torch.int32)
    per = L - 2 * R
    acc = torch.zeros(4, dtype=torch.float64, device='cuda:0')
    st = torch.zeros(1, dtype=torch.int32, device='cuda:0')
    snaps = []
    for s in range(STEPS):
        owner_lazy_step(t, walks[s].cuda(), R, K, seed=11, noise_offset=s * NW * per,
                        grad_scale=1.0 / (NW * per * 2 * R), loss_acc=acc, status=st)
        torch.cuda.synchronize()
        keep = [x.clone() for x in (t.params_in, t.m_in, t.v_in, t.last_in, t.w_out, t.m_out,
                                    t.v_out, t.last_out, t.pend_out)]
        t.flush()
        snaps.append([x[:V].cpu().clone() for x in (t.params_in[0], t.m_in, t.v_in, t.w_out,
                                                    t.m_out, t.v_out)])
        for dst, src in zip((t.params_in, t.m_in, t.v_in, t.last_in, t.w_out, t.m_out, t.v_out,
                             t.last_out, t.pend_out), keep):
            dst.copy_(src)
    return snaps, acc.cpu()


os.environ['MASTER_ADDR'] = '127.0.0.1'
os.environ['MASTER_PORT'] = '29533'
dist.init_process_group('gloo', rank=0, world_size=1)
ref, a_ref = run(False, True)
for name, (m, rm) in {'multi rows-major': (True, True), 'multi gather path': (True, False),
                      'one rank gather path': (False, False)}.items():
    got, a = run(m, rm)
    print(name, 'acc', (a - a_ref).tolist())
    for s, (x, y) in enumerate(zip(got, ref)):
        print('  step', s, ' '.join(f'{n}:{float((p - q).abs().max()):.2e}'
                                   for n, p, q in zip(('w_in', 'm_in', 'v_in', 'w_out', 'm_out',
                                                       'v_out'), x, y)))
dist.destroy_process_group()
