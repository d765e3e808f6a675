import sys
sys.path[:0] = ['.', 'x-transformers-rl_amd']
import torch
from xtrl_amd import ops
def timeit(fn, iters=50):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(iters): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3
SHAPES = [('ff2', 1024, 256, 1024), ('ff1', 1024, 1024, 256), ('qkv', 1024, 324, 256), ('head1', 1024, 1024, 512),
          ('a2', 1024, 4, 512), ('c2', 1024, 100, 512)]
if len(sys.argv) > 1 and sys.argv[1] == 'learn':   # learn-step forward shapes (16384 tokens)
    SHAPES = [('out', 16384, 256, 64), ('qkv', 16384, 324, 256), ('pred2', 16384, 18, 256), ('vals', 16384, 100, 512),
              ('a2', 16384, 4, 512), ('pd', 16384, 257, 512)]
TB = 0
if len(sys.argv) > 1 and sys.argv[1] == 'dgrad':  # learn-step input-gradient shapes (B = W [K][N] row-major)
    TB = 1
    SHAPES = [('a2', 16384, 512, 4), ('c2', 16384, 512, 100), ('pred2', 16384, 256, 18), ('pd', 16384, 512, 257),
              ('h1', 16384, 512, 1024), ('ff2', 16384, 1024, 256), ('out', 16384, 64, 256), ('qkv', 16384, 256, 324)]
for tag, M, N, K in SHAPES:
    A = torch.randn(M, K, device='cuda'); C = torch.empty(M, N, device='cuda')
    B = torch.randn(K, N, device='cuda') if TB else torch.randn(N, K, device='cuda')
    print(tag, f'{timeit(lambda: ops.gemm_ex(A, B, 0, TB, M, N, K, C)):.1f}')
