"""Host-side cost of the learn loop (cProfile over one update's learn, after a warm-up update):
where the Python time per minibatch goes when the GPU outruns the host (C2: learn idle in the trace)."""
import cProfile
import io
import pstats
import sys
import time
sys.path[:0] = ['.', 'x-transformers-rl_amd']
import torch
from bench import CONFIGS, build_learner, one_update

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else 'c2']
learner, env = build_learner(cfg, 0, use_graph=True)
one_update(learner, env, cfg['T'])
torch.cuda.synchronize()
agent = learner.agent
orig = agent.learn
prof = cProfile.Profile()
wall = {}


def learn(*a, **k):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    prof.enable()
    out = orig(*a, **k)
    prof.disable()
    wall['host'] = time.perf_counter() - t0
    torch.cuda.synchronize()
    wall['gpu_done'] = time.perf_counter() - t0
    return out


agent.learn = learn
one_update(learner, env, cfg['T'])
print(f"learn: host returns after {wall['host'] * 1e3:.1f} ms, GPU done after {wall['gpu_done'] * 1e3:.1f} ms")
s = io.StringIO()
pstats.Stats(prof, stream=s).sort_stats('tottime').print_stats(35)
print(s.getvalue())
