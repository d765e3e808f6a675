"""Fused vs two-kernel training-attention backward on the same inputs (run once per
XTRL_ATTN_FUSED_BWD value; `compare` diffs the two dumps): python tools/attn_fused_check.py run OUT.pt
/ python tools/attn_fused_check.py compare A.pt B.pt"""
import sys
from pathlib import Path
REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / 'x-transformers-rl_amd')]
import torch  # noqa: E402

if sys.argv[1] == 'run':
    from xtrl_amd import ops
    out = {}
    for (b, H, n, p) in ((3, 4, 37, 0.0), (4, 4, 128, 0.0), (4, 4, 128, 0.25), (2, 2, 10, 0.25)):
        g = torch.Generator().manual_seed(n)
        q, k, v, do = (torch.randn(b, H, n, 16, generator=g).cuda() for _ in range(4))
        lens = torch.randint(1, n + 1, (b,), generator=g).to(torch.int32)
        lens[0] = n
        lens = lens.cuda()
        qf, kf, vf = (t.clone().requires_grad_() for t in (q, k, v))
        o = ops.attention(qf, kf, vf, lens, 0.25, p, seed=3, offset=1)
        (o * do).sum().backward()
        out[(b, H, n, p)] = [t.detach().cpu() for t in (o, qf.grad, kf.grad, vf.grad)]
    torch.save(out, sys.argv[2])
else:
    A, B = torch.load(sys.argv[2]), torch.load(sys.argv[3])
    for key in A:
        diffs = [float((x - y).abs().max()) for x, y in zip(A[key], B[key])]
        print(key, 'max |diff| o, dq, dk, dv:', diffs)
