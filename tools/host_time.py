"""Is the learn phase host-bound?  One C3 update: host time to enqueue agent.learn() (no sync)
against the GPU time of the same learn (HIP events), plus a cProfile of the enqueue."""
import cProfile
import pstats
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / 'x-transformers-rl_amd')]
import torch  # noqa: E402
import bench  # noqa: E402

cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else 'c3']
learner, env = bench.build_learner(cfg, 0)
for _ in range(2):
    bench.one_update(learner, env, cfg['T'])
torch.cuda.synchronize()
agent = learner.agent
for run in range(2):
    u = agent.step
    traj, lens, genes, cum = learner.rollout_device(env, u, cfg['T'])
    fit = learner.fitness(cum, genes)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    prof = cProfile.Profile() if run == 1 else None
    e0.record()
    t0 = time.perf_counter()
    if prof:
        prof.enable()
    if run == 0:   # report every synchronizing torch operation of one learn (with its call site)
        import traceback, warnings
        torch.cuda.set_sync_debug_mode('warn')
        with warnings.catch_warnings(record=True) as caught:
            warnings.simplefilter('always')
            agent.learn(traj, lens, genes, fit, update=u)
        torch.cuda.set_sync_debug_mode(0)
        sites = {}
        for w in caught:
            sites[(w.filename, w.lineno, str(w.message)[:60])] = sites.get((w.filename, w.lineno, str(w.message)[:60]), 0) + 1
        for (f, ln, m), c in sorted(sites.items(), key=lambda kv: -kv[1]):
            print(f'sync x{c}: {f}:{ln} {m}')
    else:
        agent.learn(traj, lens, genes, fit, update=u)
    if prof:
        prof.disable()
    t1 = time.perf_counter()
    e1.record()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    agent.logs = []
    print(f'run {run}: host enqueue {1e3 * (t1 - t0):.2f} ms, until done {1e3 * (t2 - t0):.2f} ms, '
          f'GPU learn {e0.elapsed_time(e1):.2f} ms')
    if prof:
        pstats.Stats(prof).sort_stats('tottime').print_stats(18)
