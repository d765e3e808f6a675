"""Host-side cost of the host-env rollout (cProfile over one update's rollout_host, after a warm-up
update): per-wave and per-step Python time of the drop-in loop (bench.py --config lander_host)."""
import cProfile
import io
import pstats
import sys
import time
sys.path[:0] = ['.', 'x-transformers-rl_amd']
import torch
from bench import CONFIGS, build_learner, one_update

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else 'lander_host']
learner, env = build_learner(cfg, 0, use_graph=True)
one_update(learner, env, cfg['T'])
torch.cuda.synchronize()
orig = learner.rollout_host
prof = cProfile.Profile()
wall = {}


def rollout_host(*a, **k):
    t0 = time.perf_counter()
    prof.enable()
    out = orig(*a, **k)
    prof.disable()
    torch.cuda.synchronize()
    wall['s'] = time.perf_counter() - t0
    return out


learner.rollout_host = rollout_host
one_update(learner, env, cfg['T'])
eng = learner._engine[1]
print(f"rollout_host: {wall['s'] * 1e3:.1f} ms, host_times of the last wave: {eng.host_times}")
s = io.StringIO()
pstats.Stats(prof, stream=s).sort_stats('tottime').print_stats(30)
print(s.getvalue())
