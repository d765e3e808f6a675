"""Microbenchmark: training attention forward / backward at the C3 learn shape (128 episodes x
4 heads x 128 steps, dim_head 16), with and without dropout."""
import sys
from pathlib import Path
REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / 'x-transformers-rl_amd')]
import torch
from xtrl_amd import ops


def timeit(fn, iters=20):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(iters):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


b, H, n, dh = 128, 4, 128, 16
g = torch.Generator().manual_seed(0)
lens = torch.randint(1, n + 1, (b,), generator=g).to(torch.int32)
lens[0] = n
q, k, v, do = (torch.randn(b, H, n, dh, generator=g).cuda() for _ in range(4))
lens = lens.cuda()
for p in (0.0, 0.25):
    qf, kf, vf = (t.clone().requires_grad_() for t in (q, k, v))
    fwd = lambda: ops.attention(qf, kf, vf, lens, dh ** -0.5, p, seed=1, offset=0)
    t_f = timeit(fwd)
    out = fwd()
    def fb():
        o = ops.attention(qf, kf, vf, lens, dh ** -0.5, p, seed=1, offset=0)
        o.backward(do)
    t_fb = timeit(fb)
    print(f'dropout {p}: fwd {t_f:7.1f} us, fwd+bwd {t_fb:7.1f} us')
