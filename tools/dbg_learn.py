import sys, numpy as np, torch
sys.path[:0] = ['.', 'x-transformers-rl_amd', 'tests']
from test_gpu_parity import make_learner, compare_rollout
np.set_printoptions(precision=7, suppress=True, linewidth=200)
learner, env, oracle = make_learner(depth=2, gates=False, evo=False, T=10, episodes=6, batch=2, seed=5, hazard=2)
agent = learner.agent
keys = ('loss', 'actor_loss', 'critic_loss', 'autoreg_loss', 'pred_done_loss')
for u in range(2):
    traj, lens, genes, cum = learner.rollout_device(env, u, 10)
    episodes, fitness = oracle.rollout(u)
    compare_rollout(traj, lens, episodes)
    agent.learn(traj, lens, genes, None, update=u)
    oracle.learn(episodes, fitness, u)
    ours = np.array([[lg[k] for k in keys] for lg in agent.pop_logs()])
    theirs = np.array([[lg[k] for k in keys] for lg in oracle.logs]); oracle.logs = []
    print('update', u, 'lens', lens.tolist())
    print(np.concatenate([ours, ours - theirs], 1))
