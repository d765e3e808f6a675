"""Per-launch time of xtrl_dgemm (the rollout's projection GEMM) on decode shapes, graph-replayed.

    python tools/dgemm_bench.py
Each case captures 50 launches in one hipGraph and reports the replay time / 50 (graph launch
overhead included, like the rollout's captured steps)."""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / 'x-transformers-rl_amd')]

import torch  # noqa: E402

from xtrl_amd import _lib as L  # noqa: E402

CASES = [  # name, M(live), N, K, ln, act, res
    ('tiny', 16, 64, 64, False, 0, False),
    ('qkv', 1024, 260, 256, True, 0, False),
    ('qkv-440', 440, 260, 256, True, 0, False),
    ('out', 1024, 256, 64, False, 0, True),
    ('ff1', 1024, 1024, 256, True, 1, False),
    ('ff1-440', 440, 1024, 256, True, 1, False),
    ('ff1-noln', 1024, 1024, 256, False, 0, False),
    ('ff1-lnonly', 1024, 1024, 256, True, 0, False),
    ('ff1-geluonly', 1024, 1024, 256, False, 1, False),
    ('qkv-noln', 1024, 260, 256, False, 0, False),
    ('ff2', 1024, 256, 1024, False, 0, True),
    ('h1', 1024, 1024, 512, True, 2, False),
    ('h2', 1024, 104, 1024, False, 0, False),
    ('ff1-440-noln', 440, 1024, 256, False, 1, False),
    ('ff1-440-lnonly', 440, 1024, 256, True, 0, False),
    ('ff1-440-plain', 440, 1024, 256, False, 0, False),
    ('qkv-440-noln', 440, 260, 256, False, 0, False),
    ('ff2-440', 440, 256, 1024, False, 0, True),
    ('out-440', 440, 256, 64, False, 0, True),
    ('h1-440', 440, 1024, 512, True, 2, False),
    ('h1-440-noln', 440, 1024, 512, False, 2, False),
]


def main():
    dev = 'cuda'
    for name, M, N, K, ln, act, res in CASES:
        x = torch.randn(1024, K, device=dev)
        w = torch.randn(N, K, device=dev) / K ** 0.5
        b = torch.randn(N, device=dev)
        g = torch.rand(K, device=dev) + 0.5
        r = torch.randn(1024, N, device=dev)
        c = torch.empty(1024, N, device=dev)
        m = torch.tensor([M], dtype=torch.int32, device=dev)
        wp = torch.empty(L.lib().xtrl_dgemm_packed_floats(N, K), device=dev)
        L.check(L.lib().xtrl_dgemm_pack(L.ptr(w), K, N, K, L.ptr(wp), L.stream()), 'pack')

        def launch():
            L.check(L.lib().xtrl_dgemm(L.ptr(x), K, L.ptr(wp), L.ptr(b), L.ptr(g) if ln else None,
                                       min(K, 256) if ln else 0, L.ptr(r) if res else None, N, L.ptr(c), N, None,
                                       L.ptr(m), 1024, N, K, act, L.stream()), 'dgemm')
        launch()
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(50):
                launch()
        gr.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            gr.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 250
        tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
        print(f'{name:10s} M={M:5d} N={N:5d} K={K:5d}  {us:7.2f} us  {tf:6.2f} TF/s')


if __name__ == '__main__':
    main()
