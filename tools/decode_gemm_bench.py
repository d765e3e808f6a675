"""Decode-step GEMM shapes (M = envs) through xtrl_gemm_f32 with the decode epilogues; geometry is
forced with XTRL_GEMM_GEOM (tuning)."""
import os, sys
sys.path[:0] = ['.', 'x-transformers-rl_amd']
import torch
from xtrl_amd import _lib as L

lib = L.lib()
E = int(os.environ.get('E', '1024'))
d, ff, nq = 256, 1024, 260
dev = 'cuda'
R = lambda *s: torch.randn(*s, device=dev)
x = R(E, d); xn = R(E, d); W = {k: R(*s) for k, s in dict(qkv=(nq, d), out=(d, 64), ff1=(ff, d), ff2=(d, ff), h1=(4 * d, 2 * d)).items()}
b = {k: R(W[k].shape[0]) for k in W}
g = torch.ones(d, device=dev)
att, hff, y = R(E, 64), R(E, ff), torch.empty(E, 4 * d, device=dev)
acin = R(E, 2 * d)
cases = [  # tag, X, W, bias, ln, R, act, N, K
    ('qkv', xn, 'qkv', True, None, None, 0, nq, d), ('qkv+LN', x, 'qkv', True, g, None, 0, nq, d),
    ('out+res', att, 'out', False, None, x, 0, d, 64), ('ff1 gelu', xn, 'ff1', True, None, None, 1, ff, d),
    ('ff1 LN gelu', x, 'ff1', True, g, None, 1, ff, d), ('ff2+res', hff, 'ff2', True, None, x, 0, d, ff),
    ('h1 silu', acin, 'h1', True, None, None, 2, 4 * d, 2 * d)]

def launch(X, wk, bias, ln, Rr, act, N, K):
    L.check(lib.xtrl_gemm_f32(L.ptr(X), X.stride(0), L.ptr(W[wk]), K, L.ptr(b[wk]) if bias else None, L.ptr(ln),
                              L.ptr(Rr), Rr.stride(0) if Rr is not None else 0, L.ptr(y), N, None, 0, E, N, K, act,
                              L.stream()))

geom = os.environ.get('XTRL_GEMM_GEOM', 'auto')
for tag, X, wk, bias, ln, Rr, act, N, K in cases:
    f = lambda: launch(X, wk, bias, ln, Rr, act, N, K)
    f(); torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()      # GPU time per launch: 50 launches replayed from a graph
    with torch.cuda.graph(gr):
        for _ in range(50): f()
    gr.replay(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    gr.replay()
    e.record(); torch.cuda.synchronize()
    print(f'geom {geom:4s} {tag:12s} M={E} N={N} K={K}: {s.elapsed_time(e) / 50 * 1e3:7.1f} us')
