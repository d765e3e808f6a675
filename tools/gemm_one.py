"""Run one library GEMM shape repeatedly (for rocprofv3 counter passes on a single kernel).
  python tools/gemm_one.py wgrad N K M      # dW[N][K] = dY[M][N]^T X[M][K]
  python tools/gemm_one.py nn|nt M N K"""
import sys
from pathlib import Path
REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / 'x-transformers-rl_amd')]
import torch
from xtrl_amd import ops

kind = sys.argv[1]
a, b, c = (int(v) for v in sys.argv[2:5])
reps = 20
if kind == 'wgrad':
    N, K, M = a, b, c
    dy, x = torch.randn(M, N, device='cuda'), torch.randn(M, K, device='cuda')
    dw, ws = torch.zeros(N, K, device='cuda'), torch.empty(32 << 20, device='cuda')
    run = lambda: ops.wgrad(dy, x, dw, ws, beta=0.)
else:
    M, N, K = a, b, c
    A = torch.randn(M, K, device='cuda')
    B = torch.randn(K, N, device='cuda') if kind == 'nt' else torch.randn(N, K, device='cuda')
    C = torch.empty(M, N, device='cuda')
    run = lambda: ops.gemm_ex(A, B, 0, 1 if kind == 'nt' else 0, M, N, K, C)
for _ in range(reps):
    run()
torch.cuda.synchronize()
