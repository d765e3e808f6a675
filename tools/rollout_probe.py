"""Rollout timing probe (C3 by default): ms per update-rollout for the current env settings.

    python tools/rollout_probe.py [--config c3] [--reps 5]
Env: XTRL_ROLLOUT_GROUPS, XTRL_GROUP_GRAPHS, ... are read by the engine."""
import argparse
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / 'x-transformers-rl_amd')]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='c3')
    ap.add_argument('--reps', type=int, default=5)
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    torch.manual_seed(0)
    learner, env = bench.build_learner(cfg, 0)
    T = cfg['T']
    ref = None
    for u in range(2):
        traj, lens, _, _ = learner.rollout_device(env, 0, T)
    torch.cuda.synchronize()
    ref = {k: v.clone() for k, v in traj.items() if v is not None}
    ts = []
    for r in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        traj, lens, _, _ = learner.rollout_device(env, 0, T)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    same = all(torch.equal(ref[k], traj[k]) for k in ref)
    print(f'config={a.config} groups={os.environ.get("XTRL_ROLLOUT_GROUPS", "1")} '
          f'group_graphs={os.environ.get("XTRL_GROUP_GRAPHS", "0")} rollout ms: '
          f'{" ".join(f"{t:.2f}" for t in ts)}  min {min(ts):.2f}  steps {int(lens.sum())}  repeatable={same}')


if __name__ == '__main__':
    main()
