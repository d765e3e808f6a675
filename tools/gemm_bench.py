"""Microbenchmark: libxtrl_hip fp32 MFMA GEMM vs torch (hipBLASLt) on the shapes of the hot path."""
import sys, time
sys.path[:0] = ['.', 'x-transformers-rl_amd']
import torch
from xtrl_amd import ops, _lib as L

def timeit(fn, iters=20):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(iters): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3   # us

shapes = [  # (tag, M, N, K, ta, tb)
    ('dec qkv', 1024, 260, 256, 0, 0), ('dec out', 1024, 256, 64, 0, 0), ('dec ff1', 1024, 1024, 256, 0, 0),
    ('dec ff2', 1024, 256, 1024, 0, 0), ('dec head1', 1024, 1024, 512, 0, 0), ('dec vals', 1024, 100, 512, 0, 0),
    ('fwd qkv', 16384, 192, 256, 0, 0), ('fwd ff1', 16384, 1024, 256, 0, 0), ('fwd ff2', 16384, 256, 1024, 0, 0),
    ('fwd head1', 16384, 512, 512, 0, 0), ('fwd vals', 16384, 100, 512, 0, 0),
    ('dgrad ff1', 16384, 256, 1024, 0, 1), ('dgrad ff2', 16384, 1024, 256, 0, 1),
    ('wgrad ff1', 1024, 256, 16384, 1, 1), ('wgrad ff2', 256, 1024, 16384, 1, 1), ('wgrad qkv', 192, 256, 16384, 1, 1),
    ('wgrad out', 256, 64, 16384, 1, 1), ('wgrad head2', 100, 512, 16384, 1, 1),
]
for tag, M, N, K, ta, tb in shapes:
    A = torch.randn(K, M, device='cuda') if ta else torch.randn(M, K, device='cuda')
    B = torch.randn(K, N, device='cuda') if tb else torch.randn(N, K, device='cuda')
    C = torch.empty(M, N, device='cuda')
    At = A.t() if ta else A
    Bt = B if tb else B.t()
    ref = At.double() @ Bt.double()
    ops.gemm_ex(A, B, ta, tb, M, N, K, C)
    err = float((C.double() - ref).abs().max() / ref.abs().max())
    us = timeit(lambda: ops.gemm_ex(A, B, ta, tb, M, N, K, C))
    ut = timeit(lambda: torch.matmul(At, Bt, out=C))
    tf = 2 * M * N * K / us / 1e6
    print(f'{tag:10s} M={M:6d} N={N:5d} K={K:6d}  xtrl {us:8.1f} us {tf:6.1f} TF | torch {ut:8.1f} us {2*M*N*K/ut/1e6:6.1f} TF | err {err:.1e}')

print('--- weight gradients through xtrl_gemm_wgrad (split over tokens) vs torch')
ws = torch.empty(32 << 20, device='cuda')
for tag, N, K, M in [('ff1', 1024, 256, 16384), ('ff2', 256, 1024, 16384), ('proj', 260, 256, 16384),
                     ('out', 256, 64, 16384), ('head1', 1024, 768, 16384), ('head2', 100, 512, 16384),
                     ('done', 1, 512, 16384), ('pin', 256, 8, 16384)]:
    dy = torch.randn(M, N, device='cuda'); x = torch.randn(M, K, device='cuda'); dw = torch.zeros(N, K, device='cuda')
    ops.wgrad(dy, x, dw, ws, beta=0.)
    ref = dy.double().t() @ x.double()
    err = float((dw.double() - ref).abs().max() / ref.abs().max())
    us = timeit(lambda: ops.wgrad(dy, x, dw, ws, beta=0.))
    ut = timeit(lambda: torch.mm(dy.t(), x, out=dw))
    print(f'wgrad {tag:6s} N={N:5d} K={K:5d} M={M}  xtrl {us:8.1f} us {2*M*N*K/us/1e6:6.1f} TF | torch {ut:8.1f} us | err {err:.1e}')

print('--- ceiling reference: hipBLASLt bf16 GEMM with 6x the reduction length (the X6 MFMA work)')
for tag, M, N, K in [('fwd ff1', 16384, 1024, 256), ('fwd ff2', 16384, 256, 1024), ('dgrad ff1', 16384, 256, 1024),
                     ('wgrad ff1', 1024, 256, 16384), ('wgrad head1', 1024, 768, 16384)]:
    a = torch.randn(M, 6 * K, device='cuda', dtype=torch.bfloat16)
    b = torch.randn(6 * K, N, device='cuda', dtype=torch.bfloat16)
    ut = timeit(lambda: torch.matmul(a, b))
    print(f'bf16x6 {tag:12s} M={M:6d} N={N:5d} K={K:6d}: {ut:8.1f} us = {2*M*N*K/ut/1e6:6.1f} TF fp32-equivalent')
