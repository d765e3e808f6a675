"""Times the skinny weight-gradient shapes of the C3 learn step through xtrl_gemm_wgrad(_db):
run once with XTRL_WGRAD_SKINNY=0 (the 64 x 64 GEMM) and once without (k_wgrad_skinny)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'x-transformers-rl_amd'))
from xtrl_amd import _lib as L  # noqa: E402

SHAPES = [  # name, M, N, K, ldy, ldx, bias
    ('w_se', 16384, 256, 8, 517, 9, True),
    ('w_pin', 16384, 256, 8, 256, 9, False),
    ('w_pred2', 7000, 18, 256, 18, 260, True),
    ('w_pred2_T', 16384, 18, 256, 18, 260, True),
    ('w_a2', 16384, 4, 512, 4, 1024, True),
]
out = {'skinny': os.environ.get('XTRL_WGRAD_SKINNY', '1') != '0', 'us': {}}
ws = torch.empty(32 << 20, device='cuda')
for name, M, N, K, ldy, ldx, bias in SHAPES:
    dy = torch.randn(M, ldy, device='cuda')
    x = torch.randn(M, ldx, device='cuda')
    dw = torch.zeros(N, K, device='cuda')
    db = torch.zeros(N, device='cuda')

    def run():
        if bias:
            rc = L.lib().xtrl_gemm_wgrad_db(L.ptr(dy), ldy, L.ptr(x), ldx, L.ptr(dw), K, M, N, K, 1., L.ptr(ws),
                                            ws.numel(), L.ptr(db), 0, L.stream())
        else:
            rc = L.lib().xtrl_gemm_wgrad(L.ptr(dy), ldy, L.ptr(x), ldx, L.ptr(dw), K, M, N, K, 1., L.ptr(ws),
                                         ws.numel(), L.stream())
        L.check(rc, name)
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        run()
    e1.record()
    torch.cuda.synchronize()
    out['us'][name] = round(e0.elapsed_time(e1) * 1000 / 50, 2)
print(json.dumps(out))
