"""Where a scalar-host-env rollout step goes (bench --config lander_host): GPU decode step at E = 1,
eager launches vs device-timed, and the host side (action copy + sync + env step + feedback)."""
import sys, time
sys.path[:0] = ['.', 'x-transformers-rl_amd']
import torch
import bench

cfg = bench.CONFIGS['lander_host']
learner, env = bench.build_learner(cfg, 0, use_graph=False)
for _ in range(2):
    bench.one_update(learner, env, cfg['T'])
eng = learner._engine[1]
torch.cuda.synchronize()
# device time of one decode step at one live row (events), and wall with a sync per step
s, e = torch.cuda.Event(True), torch.cuda.Event(True)
N = 200
t0 = time.perf_counter()
s.record()
for t in range(N):
    eng.step(t % 50)
e.record(); torch.cuda.synchronize()
t1 = time.perf_counter()
print(f'decode step, {N} back to back: device {s.elapsed_time(e) / N * 1e3:.1f} us/step, host enqueue+run {(t1 - t0) / N * 1e6:.1f} us/step')
t0 = time.perf_counter()
for t in range(N):
    eng.step(t % 50)
    torch.cuda.synchronize()
t1 = time.perf_counter()
print(f'decode step + sync: {(t1 - t0) / N * 1e6:.1f} us/step')
t0 = time.perf_counter()
for t in range(N):
    env.step(1)
t1 = time.perf_counter()
print(f'host env step: {(t1 - t0) / N * 1e6:.1f} us')
t0 = time.perf_counter()
steps, lens = bench.one_update(learner, env, cfg['T'], phases=True)
torch.cuda.synchronize()
t1 = time.perf_counter()
ph = bench.PHASES[-1]
print(f'one update: {int(steps)} env-steps, rollout {ph[0].elapsed_time(ph[1]):.1f} ms = {ph[0].elapsed_time(ph[1]) * 1e3 / int(steps):.1f} us/step, learn {ph[1].elapsed_time(ph[2]):.1f} ms')
