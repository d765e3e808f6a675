"""Pin the oracle (oracle/ref_port.py) against golden vectors produced by the reference's own code.

The fixtures come from tests/golden/make_golden.py (run in the build container, where the
reference tree exists).  CPU only."""
import numpy as np
import pytest
import torch

from oracle import ref_port as R
from oracle import thirdparty as tp


def T(a):
    return torch.from_numpy(np.asarray(a))


def close(a, b, rtol=1e-5, atol=1e-6):
    a = a.detach().cpu().numpy() if torch.is_tensor(a) else np.asarray(a)
    np.testing.assert_allclose(a, np.asarray(b), rtol=rtol, atol=atol)


def test_gae(golden):
    g = golden('gae')
    close(R.calc_gae(T(g['rewards']), T(g['values']), T(g['masks']).float()), g['returns'], 0, 0)
    close(R.calc_gae(T(g['rewards']), T(g['values']), T(g['masks']).float(), 0.9, 0.5), g['returns_g09_l05'], 0, 0)


def test_rsnorm(golden):
    g = golden('rsnorm')
    rs = R.RSNormState(6)
    for i in range(4):
        out = rs.train_call(T(g[f'in{i}']))
        close(out, g[f'out{i}'], 1e-6, 1e-6)
        close(rs.mean, g['means'][i], 1e-6, 1e-7)
        close(rs.var, g['variances'][i], 1e-6, 1e-7)
        assert rs.step == int(g['steps'][i])
    close(rs.apply(T(g['eval_in'])), g['eval_out'], 1e-6, 1e-6)


def test_normalize_and_distributions(golden):
    g = golden('dists')
    t, m = T(g['t']), T(g['mask'])
    close(R.normalize(t, m), g['norm_masked'], 1e-6, 1e-6)
    close(R.normalize(t), g['norm_all'], 1e-6, 1e-6)
    close(R.normalize(t, torch.zeros_like(m)), g['norm_empty'], 0, 0)
    raw, a = T(g['raw']), T(g['actions'])
    probs, _ = R.categorical_logits(raw)
    close(probs, g['probs'], 1e-6, 1e-7)
    close(R.discrete_log_prob(raw, a), g['log_prob'], 1e-6, 1e-6)
    close(R.discrete_entropy(raw), g['entropy'], 1e-6, 1e-6)
    craw, cval = T(g['craw']), T(g['cval'])
    close(R.continuous_log_prob(craw, cval, True), g['c_lp_squash'], 1e-5, 1e-5)
    close(R.continuous_log_prob(craw, cval, False), g['c_lp'], 1e-5, 1e-5)
    close(R.continuous_entropy(craw), g['c_entropy'], 1e-6, 1e-6)
    mean, var = R.continuous_params(craw)
    close(torch.stack((mean, var)), g['c_mean_var'], 1e-6, 1e-6)


@pytest.mark.parametrize('tag,cont', [('d', False), ('c', True)])
def test_actor_critic_losses(golden, tag, cont):
    g = golden('losses')
    cfg = R.ModelConfig(5, 3, 32, continuous=cont, squash=True, reward_range=(-2., 2.))
    hl = tp.HLGaussLoss(-2., 2., 100, clamp_to_range=True)
    lens = T(g[f'{tag}_lens'])
    mask = torch.arange(7)[None] < lens[:, None]
    al = R.actor_loss(cfg, hl, T(g[f'{tag}_raw']), T(g[f'{tag}_actions']), T(g[f'{tag}_old_lp']),
                      T(g[f'{tag}_returns']), T(g[f'{tag}_old_values']), mask)
    close(al, g[f'{tag}_actor'], 1e-5, 1e-6)
    cl = R.critic_loss(cfg, hl, T(g[f'{tag}_values']), T(g[f'{tag}_returns']), T(g[f'{tag}_old_values']))
    close(cl, g[f'{tag}_critic'], 1e-6, 1e-6)


def test_world_model_losses(golden):
    g = golden('losses')
    close(R.autoregressive_loss(T(g['pred']), T(g['real'])), g['wm_loss'], 1e-6, 1e-6)
    close(R.done_loss(T(g['done_pred']), T(g['dones'])), g['done_loss'], 1e-6, 1e-6)


def _model_from_fixture(g):
    cfg = R.ModelConfig(6, 4, 32, depth=2, reward_range=(-2., 2.), evolutionary=True, dim_gene=8,
                        frac_head_grad=0.3, gate_values=True, value_residual=True, learned_mix=True)
    m = R.OracleWMAC(cfg)
    sd = {k[3:]: T(g[k]) for k in g.files if k.startswith('sd.')}
    missing = m.load_state_dict(sd, strict=True)
    return m


def test_model_forward_and_grads(golden):
    g = golden('model_forward')
    m = _model_from_fixture(g)
    m.train()
    lens = T(g['lens'])
    mask = torch.arange(9)[None] < lens[:, None]
    raw, values, pred, dones, _ = m(T(g['state']), actions=T(g['prev']), rewards=T(g['rewards']),
                                    next_actions=T(g['actions']), latent_gene=T(g['latent']), mask=mask)
    close(raw, g['raw'], 1e-5, 1e-6)
    close(values, g['values'], 1e-5, 1e-6)
    close(pred, g['state_pred'], 1e-5, 1e-6)
    close(dones, g['dones'], 1e-5, 1e-6)
    (raw.pow(2).sum() + values.sum() * 0.5 + pred.sum() + dones.sum()).backward()
    for name, p in m.named_parameters():
        key = f'grad.{name}'
        if key in g.files:
            close(p.grad, g[key], 1e-4, 1e-6)
    m.eval()
    cache = None
    with torch.no_grad():
        for t in range(5):
            r, v, _, _, cache = m(T(g['state'])[:1, t:t + 1], rewards=T(g['rewards'])[0, t],
                                  actions=T(g['prev'])[:1, t:t + 1], latent_gene=T(g['latent'])[:1], cache=cache)
            close(r[0, 0], g['dec_raw'][t], 1e-5, 1e-6)
            close(v[0, 0], g['dec_values'][t], 1e-5, 1e-6)


def test_evolve(golden):
    g = golden('evolve')
    for case in range(3):
        islands, per, sel, tourn, steps = (int(x) for x in g[f'c{case}_cfg'])
        genes = T(g[f'c{case}_genes0'])
        for s in range(steps):
            torch.manual_seed(1000 + 10 * case + s)
            genes, selected = R.evolve(genes, T(g[f'c{case}_fitnesses'][s]), islands, sel, tourn, step=s)
            close(genes, g[f'c{case}_genes'][s], 1e-6, 1e-6)
            np.testing.assert_array_equal(selected.numpy(), g[f'c{case}_selected'][s])


def _learner_from_fixture(g):
    seed, S, A, Tm, depth, gates, evo, episodes, batch, updates, hz, gdim = (int(x) for x in g['cfg'])
    c = R.LearnerConfig(S, A, (-2., 2.), depth=depth, gate_values=bool(gates), value_residual=bool(gates),
                        learned_mix=bool(gates), evolutionary=bool(evo), evolve_every=1, evolve_after_step=0,
                        gene_pool=dict(dim=gdim, num_genes_per_island=3, num_selected=2, tournament_size=2),
                        max_timesteps=Tm, batch_size=batch, num_episodes_per_update=episodes,
                        sim_mode=str(g['mode']), hazard_log2=hz, reward_dropout=float(g['reward_dropout']),
                        seed=seed)
    sd = {k[5:]: T(g[k]) for k in g.files if k.startswith('init.')}
    return R.OracleLearner(c, init_state_dict=sd, genes=T(g['init_genes']) if evo else None), updates


@pytest.mark.parametrize('name', ['learner_readme', 'learner_lander_evo'])
def test_learner_end_to_end(golden, name):
    g = golden(name)
    L, updates = _learner_from_fixture(g)
    for u in range(updates):
        episodes, fitness = L.rollout(u)
        lens = torch.tensor([ep['len'] for ep in episodes])
        np.testing.assert_array_equal(lens.numpy(), g[f'u{u}.lens'])
        n = int(lens.max())
        acts = torch.nn.utils.rnn.pad_sequence([torch.stack([m[1] for m in ep['mem']]) for ep in episodes], True)
        np.testing.assert_array_equal(acts.numpy(), g[f'u{u}.actions'])
        lp = torch.nn.utils.rnn.pad_sequence([torch.stack([m[2] for m in ep['mem']]) for ep in episodes], True)
        close(lp, g[f'u{u}.logp'], 1e-5, 1e-6)
        vals = torch.nn.utils.rnn.pad_sequence([torch.stack([m[5] for m in ep['mem']]) for ep in episodes], True)
        close(vals, g[f'u{u}.values'], 1e-5, 1e-5)
        if f'u{u}.fitness' in g.files:
            close(fitness, g[f'u{u}.fitness'], 1e-5, 1e-5)
        L.learn(episodes, fitness, u)
    keys = list(g['log_keys'])
    ours = np.array([[lg[k] for k in keys] for lg in L.logs])
    np.testing.assert_allclose(ours, g['logs'], rtol=1e-4, atol=1e-6)
    for k, p in L.model.state_dict().items():
        close(p, g[f'final.{k}'], 1e-4, 1e-6)
    for k, p in L.ema.ema_model.state_dict().items():
        close(p, g[f'ema.{k}'], 1e-4, 1e-6)
    close(L.rsnorm.mean, g['rs_mean'], 1e-5, 1e-6)
    close(L.rsnorm.var, g['rs_var'], 1e-5, 1e-6)
    assert L.rsnorm.step == int(g['rs_step'])
    if 'final_genes' in g.files:
        close(L.genes, g['final_genes'], 1e-5, 1e-6)
