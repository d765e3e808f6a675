"""Training attention fwd / fwd+bwd with and without dropout at the C3 (b 128, n 128) and C2 (b 32,
n 500) learn shapes, dh 16 x 4 heads: the share of the Philox keep bits in the attention time."""
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


for (b, n, lo) in ((128, 128, 1), (32, 500, 300)):
    H, dh = 4, 16
    g = torch.Generator().manual_seed(0)
    lens = torch.randint(lo, n + 1, (b,), generator=g).to(torch.int32)
    lens[0] = n
    q, k, v, do = (torch.randn(b, H, n, dh, generator=g).cuda() for _ in range(4))
    lens = lens.cuda()
    for p in (0.25, 0.0, 0.25, 0.0):
        qf, kf, vf = (t.clone().requires_grad_() for t in (q, k, v))
        fwd = lambda: ops.attention(qf, kf, vf, lens, dh ** -0.5, p, seed=1, offset=0)
        t_f = timeit(fwd)
        def fb():
            o = ops.attention(qf, kf, vf, lens, dh ** -0.5, p, seed=1, offset=0)
            o.backward(do)
        t_fb = timeit(fb)
        print(f'b {b} n {n}: dropout {p}: fwd {t_f:7.1f} us, fwd+bwd {t_fb:7.1f} us')
