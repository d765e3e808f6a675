"""Gradient error of the fractal-body learn step against fp32 and fp64 oracles (diagnostic).

    python tools/fractal_grad_probe.py
For each minibatch of one update: max |g_gpu - g_fp64| / scale and max |g_fp32 - g_fp64| / scale,
with the parameter that attains it."""
import copy
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / 'x-transformers-rl_amd'), str(REPO / 'tests')]

import torch  # noqa: E402

from oracle import ref_port as R  # noqa: E402
from test_gpu_parity import make_learner, oracle_minibatch_tensors  # noqa: E402


def main(levels=2, evo=False, cont=False):
    learner, env, oracle = make_learner(depth=2, gates=False, evo=evo, cont=cont, T=10, episodes=6, batch=2, seed=5,
                                        hazard=2, fractal_levels=levels)
    agent = learner.agent
    c = oracle.c
    traj, lens, genes, cum = learner.rollout_device(env, 0, 10)
    lens_c = lens.cpu()
    eps = []
    for i in range(6):
        n = int(lens_c[i])
        acts = traj['actions_f'][i, :n].cpu() if cont else traj['actions'][i, :n].cpu().long()
        eps.append(dict(mem=list(zip(traj['states'][i, :n].cpu(), acts, traj['logp'][i, :n].cpu(),
                                     traj['rewards'][i, :n].cpu(), traj['bounds'][i, :n].cpu().bool(),
                                     traj['values'][i, :n].cpu())), len=n, gene=0))
    states, actions, old_lp, rewards, bounds, values, elens, egenes = oracle_minibatch_tensors(eps)
    returns = R.calc_gae(rewards, oracle.model.hl(values), (~bounds).float(), c.gamma, c.lam)

    def grads(model, dt, idx, epoch, mbi):
        rs = R.RSNormState(c.state_dim + 1)
        rs.mean, rs.var = agent.rs_mean.cpu().to(dt), agent.rs_var.cpu().to(dt)
        f = lambda t: t.to(dt) if t.is_floating_point() else t   # noqa: E731
        mb = R.Minibatch(f(states[idx]), f(actions[idx]), f(rewards[idx]), f(old_lp[idx]), f(returns[idx]),
                         f(values[idx]), bounds[idx], egenes[idx], elens[idx])
        model.train()
        model.zero_grad()
        keep = R.reward_coin(c.seed, 0, epoch, mbi, c.reward_dropout)
        loss, _, _, _ = R.minibatch_loss(model, rs, mb, None, c.weights, keep)
        loss.backward()
        return float(loss), {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}

    def probe(epoch, mbi, idx, loss, stats):
        idx = idx.cpu()
        sd = {k: v.detach().cpu() for k, v in agent.model.state_dict().items()}
        oracle.model.load_state_dict(sd)
        m64 = copy.deepcopy(oracle.model).double()
        l32, g32 = grads(oracle.model, torch.float32, idx, epoch, mbi)
        l64, g64 = grads(m64, torch.float64, idx, epoch, mbi)
        gpu = dict(zip(agent.flat.names, (p.grad.detach().cpu().double() for p in agent.flat.params)))
        scale = max(float(g.abs().max()) for g in g64.values())
        e_gpu = max((float((gpu[n] - g).abs().max()), n) for n, g in g64.items())
        e_32 = max((float((g32[n].double() - g).abs().max()), n) for n, g in g64.items())
        print(f'epoch {epoch} mb {mbi}: loss gpu {float(loss):.7f} f32 {l32:.7f} f64 {l64:.7f} | '
              f'grad err / scale: gpu {e_gpu[0] / scale:.2e} ({e_gpu[1]})  f32 {e_32[0] / scale:.2e} ({e_32[1]})')

    agent.learn(traj, lens, genes, None, update=0, probe=probe)


if __name__ == '__main__':
    main()
    main(3, cont=True)
