"""Phase times of the row-resident decode step (xtrl_row_stamps) at the lander_host shape (d 48,
depth 4, one live row) for a few positions t: where the ~65 us of a host-env decode step go."""
import ctypes as C
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'x-transformers-rl_amd')]
import numpy as np
import torch
import bench
from xtrl_amd import _lib as L

cfg = dict(bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else 'lander_host'])
learner, env = bench.build_learner(cfg, 0, use_graph=False)
bench.one_update(learner, env, cfg['T'])
eng = learner._engine[1]
lib = L.lib()
Lyr = eng.c.depth
names = ['compact', 'embed'] + [f'L{l}.{p}' for l in range(Lyr) for p in ('ln1', 'qkv', 'attn', 'out', 'ln2', 'ff1', 'ff2')] + \
        ['lnf', 'h1', 'h2', 'sample']
buf = (C.c_uint64 * 2048)()
rate = C.c_int64()
torch.cuda.synchronize()
for t in (1, 64, 256, 448):
    if t >= eng.T:
        continue
    eng.alive[:1].fill_(1)
    eng.alive[1:].zero_()
    lib.xtrl_row_stamps(1, buf, 0, C.byref(rate))
    for rep in range(3):
        eng.step(t, True)
        torch.cuda.synchronize()
    cap = lib.xtrl_row_stamps(0, buf, 2048, C.byref(rate))
    st = np.array(buf[:len(names) + 1], dtype=np.float64)
    cy = np.array(buf[cap:cap + len(names) + 1], dtype=np.float64)
    us = np.diff(st) / rate.value * 1e6
    tot = (st[-1] - st[0]) / rate.value * 1e6
    ghz = (cy[-1] - cy[0]) / (tot * 1e3)
    print(f't={t}: total {tot:.1f} us, shader clock {ghz:.2f} GHz  ' + '  '.join(f'{n} {u:.2f}' for n, u in zip(names, us)))

# the step's device time with stamping off and on (events over 200 back-to-back launches at t = 64)
for on in (0, 1, 0):
    lib.xtrl_row_stamps(on, buf, 0, C.byref(rate))
    eng.alive[:1].fill_(1)
    eng.alive[1:].zero_()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(200):
        eng.step(64, True)
    b.record()
    torch.cuda.synchronize()
    print(f'stamping {on}: {a.elapsed_time(b) / 200 * 1e3:.1f} us/step')
lib.xtrl_row_stamps(0, buf, 0, C.byref(rate))
