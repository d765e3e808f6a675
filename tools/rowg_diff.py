"""Rollout trajectory of the failing gradient-parity configuration under the current XTRL_ROW_G,
saved to gpurun_out/traj_g<G>.npz; `python tools/rowg_diff.py cmp` compares two saves field by field
(max |diff|, positions past each row's length that are non-zero)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'tests'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'x-transformers-rl_amd'))
if sys.argv[1:] == ['cmp']:
    a, b = np.load('gpurun_out/traj_g1.npz'), np.load('gpurun_out/traj_g4.npz')
    lens = a['lens']
    print('lens equal', np.array_equal(a['lens'], b['lens']), a['lens'].tolist(), b['lens'].tolist())
    for k in a.files:
        x, y = a[k], b[k]
        d = np.abs(x.astype(np.float64) - y.astype(np.float64))
        print(k, x.shape, 'max|diff|', float(d.max()) if d.size else 0., 'n_diff', int((d > 0).sum()))
        if x.ndim >= 2 and k != 'lens' and not k.startswith('flat'):
            for name, t in (('g1', x), ('g4', y)):
                pad = [float(np.abs(t[i, lens[i]:]).max()) if lens[i] < t.shape[1] else 0. for i in range(t.shape[0])]
                if max(pad) > 0:
                    print('   non-zero padding', name, pad)
    sys.exit(0)
import torch  # noqa: E402
import test_gpu_parity as P  # noqa: E402
learner, env, oracle = P.make_learner(depth=2, gates=False, evo=False, cont=False, T=10, episodes=6, batch=2, seed=5,
                                      hazard=2)
out = {}
for u in range(2):
    traj, lens, genes, cum = learner.rollout_device(env, u, 10)
    torch.cuda.synchronize()
    for k, v in traj.items():
        if v is not None:
            out[f'{k}{u}'] = v.cpu().numpy()
    out[f'lens{u}'] = lens.cpu().numpy()
    learner.agent.learn(traj, lens, genes, learner.fitness(cum, genes), update=u)
    out[f'flat{u}'] = learner.agent.flat.flat.detach().cpu().numpy()
out['lens'] = out['lens0']
np.savez(f"gpurun_out/traj_g{os.environ.get('XTRL_ROW_G', '4')}.npz", **out)
print('saved', sorted(out))
