"""Generate the golden vectors by running the REFERENCE's own code in this container.

Runs only where /root/reference exists (never on the GPU box).  The reference is pure Python;
its un-vendored third-party imports (einx, x_transformers, assoc_scan, hl_gauss_pytorch,
ema_pytorch, adam_atan2_pytorch — SURVEY §8c) are satisfied with the restatements in
oracle/thirdparty.py, so the vectors pin the reference's OWN arithmetic and glue
(x_transformers_rl.py, evolution.py) while the third-party maths stays parity-unpinned.

Output: small .npz files (data only, no pickles) next to this script.  Re-run with
    python tests/golden/make_golden.py
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
REF = Path(os.environ.get('XTRL_REFERENCE', '/root/reference')) / 'x_transformers_rl'
sys.path.insert(0, str(REPO))
os.environ.setdefault('TQDM_DISABLE', '1')

from oracle import thirdparty as tp                                          # noqa: E402
from oracle.philox import (FIELD_SAMPLE, SynthSim, epoch_permutation, evolve_seed,  # noqa: E402
                           philox_uniform, reward_coin)


def load_reference():
    """Import distributed.py / evolution.py / x_transformers_rl.py by path with stand-ins."""
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m
    mod('einx', multiply=tp.einx.multiply, less=tp.einx.less, where=tp.einx.where)
    mod('assoc_scan', AssocScan=tp.AssocScan)
    mod('hl_gauss_pytorch', HLGaussLoss=tp.HLGaussLoss)
    mod('x_transformers', Decoder=tp.Decoder, ContinuousTransformerWrapper=tp.ContinuousTransformerWrapper,
        Attention=tp.XAttention, FeedForward=tp.FeedForward)
    mod('ema_pytorch', EMA=tp.EMA)
    mod('adam_atan2_pytorch', AdoptAtan2=tp.AdoptAtan2)
    pkg = mod('x_transformers_rl')
    pkg.__path__ = [str(REF)]
    out = {}
    for name in ('distributed', 'evolution', 'x_transformers_rl', 'fractal_rl'):
        spec = importlib.util.spec_from_file_location(f'x_transformers_rl.{name}', REF / f'{name}.py')
        m = importlib.util.module_from_spec(spec)
        sys.modules[spec.name] = m
        spec.loader.exec_module(m)
        out[name] = m
    return out


def save(name, **arrays):
    arrays = {k: (v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v)) for k, v in arrays.items()}
    np.savez(HERE / f'{name}.npz', **arrays)
    print(f'wrote {name}.npz  ({sum(a.nbytes for a in arrays.values()) / 1024:.1f} KiB)')


def sd_arrays(prefix, sd):
    return {f'{prefix}{k}': v for k, v in sd.items()}


# --------------------------------------------------------------------------------------------


def gen_gae(X):
    g = torch.Generator().manual_seed(1)
    b, n = 6, 37
    rewards = torch.randn(b, n, generator=g)
    values = torch.randn(b, n, generator=g)
    masks = torch.rand(b, n, generator=g) > 0.1
    masks[0] = True
    masks[1, -1] = False
    ret = X.calc_gae(rewards, values, masks, gamma=0.99, lam=0.95, use_accelerated=False)
    ret2 = X.calc_gae(rewards, values, masks, gamma=0.9, lam=0.5, use_accelerated=False)
    save('gae', rewards=rewards, values=values, masks=masks, returns=ret, returns_g09_l05=ret2)


def gen_rsnorm(X):
    g = torch.Generator().manual_seed(2)
    rs = X.RSNorm(6)
    rs.train()
    inputs, outs, means, variances, steps = [], [], [], [], []
    for k, shape in enumerate([(7, 6), (3, 5, 6), (1, 6), (11, 6)]):
        x = torch.randn(*shape, generator=g) * (k + 1) + k
        outs.append(rs(x).reshape(-1, 6))
        inputs.append(x.reshape(-1, 6))
        means.append(rs.running_mean.clone())
        variances.append(rs.running_variance.clone())
        steps.append(rs.step.clone())
    rs.eval()
    x = torch.randn(5, 6, generator=g)
    ev = rs(x)
    save('rsnorm', **{f'in{i}': a for i, a in enumerate(inputs)}, **{f'out{i}': a for i, a in enumerate(outs)},
         means=torch.stack(means), variances=torch.stack(variances), steps=torch.stack(steps),
         eval_in=x, eval_out=ev)


def gen_normalize_and_dists(X):
    g = torch.Generator().manual_seed(3)
    t = torch.randn(4, 9, generator=g)
    mask = torch.rand(4, 9, generator=g) > 0.4
    empty = torch.zeros(4, 9, dtype=torch.bool)
    raw = torch.randn(10, 4, generator=g) * 3
    raw[0] = torch.tensor([50., -50., 0., 1.])        # exercise the eps clamp of Categorical
    acts = torch.randint(0, 4, (10,), generator=g)
    d = X.Discrete(raw)
    craw = torch.randn(10, 6, generator=g) * 2
    cval = torch.rand(10, 3, generator=g) * 1.8 - 0.9
    c_sq = X.Continuous(craw, squash=True)
    c_ns = X.Continuous(craw, squash=False)
    save('dists', t=t, mask=mask, norm_masked=X.normalize(t, mask), norm_all=X.normalize(t),
         norm_empty=X.normalize(t, empty), raw=raw, actions=acts, probs=d.probs, log_prob=d.log_prob(acts),
         entropy=d.entropy(), craw=craw, cval=cval, c_lp_squash=c_sq.log_prob(cval), c_lp=c_ns.log_prob(cval),
         c_entropy=c_ns.entropy(), c_mean_var=c_ns.mean_variance)


def build_wmac(X, *, S, A, d, depth, continuous, evolutionary, G, gates):
    wm = dict(attn_dim_head=16, heads=4, depth=depth)
    if gates:
        wm.update(attn_gate_values=True, add_value_residual=True, learned_value_residual_mix=True)
    transformer = tp.ContinuousTransformerWrapper(
        dim_in=S, dim_out=None, max_seq_len=64, probabilistic=True,
        attn_layers=tp.Decoder(dim=d, rotary_pos_emb=True, attn_dropout=0., ff_dropout=0., verbose=False, **wm))
    return X.WorldModelActorCritic(transformer=transformer, num_actions=A, critic_dim_pred=100,
                                   critic_min_max_value=(-2., 2.), state_dim=S, continuous_actions=continuous,
                                   squash_continuous=True, frac_actor_critic_head_gradient=0.3,
                                   entropy_weight=0.01, evolutionary=evolutionary, dim_latent_gene=G)


def gen_losses(X):
    g = torch.Generator().manual_seed(4)
    torch.manual_seed(4)
    out = {}
    for tag, cont in (('d', False), ('c', True)):
        m = build_wmac(X, S=5, A=3, d=32, depth=1, continuous=cont, evolutionary=False, G=None, gates=False)
        b, n, B = 3, 7, 100
        lens = torch.tensor([7, 4, 1])
        mask = torch.arange(n)[None] < lens[:, None]
        raw = torch.randn(b, n, 6 if cont else 3, generator=g)
        acts = (torch.rand(b, n, 3, generator=g) * 1.8 - 0.9) if cont else torch.randint(0, 3, (b, n), generator=g)
        old_lp = torch.randn(b, n, *((3,) if cont else ()), generator=g) * 0.3 - 1.
        returns = torch.randn(b, n, generator=g)
        old_values = torch.randn(b, n, B, generator=g)
        values = torch.randn(b, n, B, generator=g)
        out.update({f'{tag}_raw': raw, f'{tag}_actions': acts, f'{tag}_old_lp': old_lp, f'{tag}_returns': returns,
                    f'{tag}_old_values': old_values, f'{tag}_values': values, f'{tag}_lens': lens,
                    f'{tag}_actor': m.compute_actor_loss(raw, acts, old_lp, returns, old_values, mask=mask),
                    f'{tag}_critic': m.compute_critic_loss(values, returns, old_values)})
    pred = torch.stack((torch.randn(3, 7, 6, generator=g), torch.rand(3, 7, 6, generator=g) + 1e-7))
    real = torch.randn(3, 7, 6, generator=g)
    done_pred = torch.rand(3, 7, generator=g)
    dones = torch.rand(3, 7, generator=g) > 0.7
    out.update(pred=pred, real=real, wm_loss=m.compute_autoregressive_loss(pred, real), done_pred=done_pred,
               dones=dones, done_loss=m.compute_done_loss(done_pred, dones))
    save('losses', **out)


def gen_model_forward(X):
    torch.manual_seed(5)
    g = torch.Generator().manual_seed(5)
    S, A, d, G = 6, 4, 32, 8
    m = build_wmac(X, S=S, A=A, d=d, depth=2, continuous=False, evolutionary=True, G=G, gates=True)
    with torch.no_grad():   # make the gate / mix paths non-trivial (their init is constant)
        for name, p in m.named_parameters():
            if 'to_v_gate' in name or 'to_value_residual_mix' in name:
                p.copy_(torch.randn(p.shape, generator=g) * 0.3)
    m.train()
    b, n = 3, 9
    state = torch.randn(b, n, S, generator=g)
    actions = torch.randint(0, A, (b, n), generator=g)
    prev = torch.cat((torch.full((b, 1), -1), actions[:, :-1]), dim=1)
    rewards = torch.randn(b, n, generator=g)
    lens = torch.tensor([9, 5, 2])
    mask = torch.arange(n)[None] < lens[:, None]
    latent = torch.nn.functional.normalize(torch.randn(b, G, generator=g), dim=-1)
    m.reward_dropout.p = 0.
    raw, values, state_pred, dones, _ = m(state, rewards=rewards, actions=prev, latent_gene=latent,
                                         next_actions=actions, mask=mask)
    (raw.pow(2).sum() + values.sum() * 0.5 + state_pred.sum() + dones.sum()).backward()
    grads = {f'grad.{k}': p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}
    # cached single-token decode, as the rollout drives it (xtrl.py:1250-1280), batch 1
    m.eval()
    cache, dec_raw, dec_val = None, [], []
    with torch.no_grad():
        for t in range(5):
            r, v, _, _, cache = m(state[:1, t:t + 1], rewards=rewards[0, t], actions=prev[:1, t:t + 1],
                                  latent_gene=latent[:1], cache=cache)
            dec_raw.append(r[0, 0])
            dec_val.append(v[0, 0])
    save('model_forward', **sd_arrays('sd.', m.state_dict()), **grads, state=state, actions=actions, prev=prev,
         rewards=rewards, lens=lens, latent=latent, raw=raw, values=values, state_pred=state_pred, dones=dones,
         dec_raw=torch.stack(dec_raw), dec_values=torch.stack(dec_val))


def gen_evolve(X, E):
    out = {}
    for case, (islands, per, sel, tourn, steps) in enumerate([(1, 3, 2, 2, 3), (1, 8, 4, 2, 2), (2, 6, 3, 3, 12)]):
        torch.manual_seed(100 + case)
        pool = E.LatentGenePool(dim=8, num_genes_per_island=per, num_selected=sel, tournament_size=tourn,
                                num_islands=islands, migrate_genes_every=10)
        g0 = pool.genes.detach().clone()
        fits, genes_after, selected = [], [], []
        try:
            for s in range(steps):
                f = torch.randn(pool.num_genes)
                torch.manual_seed(1000 + 10 * case + s)
                selected.append(pool.evolve_(f))
                fits.append(f)
                genes_after.append(pool.genes.detach().clone())
        except TypeError as err:   # evolution.py:148 slices with a float when migration fires
            print(f'evolve case {case}: reference raised at step {len(fits)}: {err}')
        out.update({f'c{case}_genes0': g0, f'c{case}_fitnesses': torch.stack(fits),
                    f'c{case}_genes': torch.stack(genes_after), f'c{case}_selected': torch.stack(selected),
                    f'c{case}_cfg': torch.tensor([islands, per, sel, tourn, len(fits)])})
    save('evolve', **out)


def _perturb(module, seed):
    """Non-trivial weights for a fixture: every parameter redrawn (LayerNorm gains around 1), so the
    level embeddings, the global-state init and the norms all matter."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in module.named_parameters():
            scale = 1.0 / p.shape[-1] ** 0.5 if p.ndim > 1 else 0.3
            base = 1.0 if ('norm' in name and name.endswith('weight')) else 0.0
            p.copy_(torch.randn(p.shape, generator=g) * scale + base)


def gen_fractal(Fr):
    """The reference's own fractal modules (fractal_rl.py), eval mode, x-transformers Attention /
    FeedForward restated (oracle/thirdparty.py XAttention / FeedForward):
      FractalLevelEmbedding.forward            :63-67
      FractalProcessingBlock.forward           :116-132 (with and without the global state, ragged mask)
      FractalEncoder.forward                   :276-346 (separate / shared / hypernetwork blocks)
      FractalWorldModelActorCritic.forward     :548-619 (discrete + gene, continuous; n = 8 and n = 1)"""
    torch.manual_seed(21)
    g = torch.Generator().manual_seed(21)
    out = {}
    le = Fr.FractalLevelEmbedding(24, 5)
    _perturb(le, 1)
    out.update(sd_arrays('le.', le.state_dict()))
    out['le.out'] = torch.stack([le(i) for i in range(5)])

    blk = Fr.FractalProcessingBlock(32, heads=4, dim_head=8, dropout=0.1).eval()
    _perturb(blk, 2)
    x = torch.randn(3, 7, 32, generator=g)
    gs = torch.randn(3, 1, 32, generator=g)
    mask = torch.arange(7)[None] < torch.tensor([7, 4, 1])[:, None]
    with torch.no_grad():
        out.update(sd_arrays('blk.', blk.state_dict()))
        out.update({'blk.x': x, 'blk.g': gs, 'blk.mask': mask, 'blk.out': blk(x, gs, mask),
                    'blk.out_nomask': blk(x, gs), 'blk.out_noglobal': blk(x, None, mask)})

    xs = torch.randn(3, 9, 6, generator=g)
    emask = torch.arange(9)[None] < torch.tensor([9, 5, 1])[:, None]
    out.update({'enc.x': xs, 'enc.mask': emask})
    for tag, kw in (('sep', {}), ('share', dict(share_weights=True)), ('hyper', dict(use_hypernetwork=True))):
        enc = Fr.FractalEncoder(6, embed_dim=32, num_levels=3, heads=4, dim_head=8, dropout=0.1, **kw).eval()
        _perturb(enc, 3)
        with torch.no_grad():
            agg, levels = enc(xs, mask=emask if tag == 'sep' else None, return_all_levels=True)
        out.update(sd_arrays(f'enc_{tag}.', enc.state_dict()))
        out[f'enc_{tag}.agg'] = agg
        out[f'enc_{tag}.levels'] = torch.stack(levels)

    for tag, cont, evo in (('wm_d', False, True), ('wm_c', True, False)):
        wm = Fr.FractalWorldModelActorCritic(6, 4, 100, (-2., 2.), embed_dim=32, num_fractal_levels=2, heads=4,
                                             dim_head=8, dropout=0.1, continuous_actions=cont, squash_continuous=cont,
                                             evolutionary=evo, dim_latent_gene=8 if evo else None).eval()
        _perturb(wm, 4)
        out.update(sd_arrays(f'{tag}.', wm.state_dict()))
        for n in (8, 1):
            st = torch.randn(3, n, 6, generator=g)
            nxt = torch.rand(3, 4, generator=g) * 1.8 - 0.9 if cont else torch.tensor([2, -1, 0])
            lat = torch.nn.functional.normalize(torch.randn(3, 8, generator=g), dim=-1) if evo else None
            with torch.no_grad():
                raw, val, sp, dn, cache = wm(st, next_actions=nxt, latent_gene=lat)
            p = f'{tag}.n{n}.'
            out.update({p + 'state': st, p + 'next_actions': nxt, p + 'raw': raw, p + 'values': val,
                        p + 'state_pred': sp, p + 'dones': dn, p + 'levels': torch.stack(cache['fractal_levels'])})
            if evo:
                out[p + 'latent'] = lat
    save('fractal', **out)


# --------------------------------------------------------------------------------------------
# full Learner: the reference's own rollout + learn, with the shared-uniform protocol patched in
# --------------------------------------------------------------------------------------------


class Harness:
    def __init__(self, seed, n_genes, S, A, mode, hazard_log2):
        self.seed, self.n_genes, self.S, self.A = seed, n_genes, S, A
        self.mode, self.hazard_log2 = mode, hazard_log2
        self.update, self.slot, self.t = 0, -1, 0
        self.epoch, self.mb = 0, 0
        self.p_reward = 0.5
        self.logs, self.learn_inputs = [], []


def gen_learner(X, name, *, seed, S, A, T, depth, gates, evolutionary, episodes, batch, updates, mode,
                hazard_log2, reward_dropout, gene_dim=8):
    H = Harness(seed, 3 if evolutionary else 1, S, A, mode, hazard_log2)
    H.p_reward = reward_dropout

    class Sim:
        def reset(self, seed=None):
            H.slot += 1
            H.t = 0
            self.sim = SynthSim(H.seed, H.update, H.slot // H.n_genes, H.S, H.A, H.mode, H.hazard_log2)
            return self.sim.reset()

        def step(self, actions):
            return self.sim.step(np.asarray(actions))

    def icdf_sample(self):
        u = torch.from_numpy(philox_uniform(H.seed, H.update, H.slot, H.t, FIELD_SAMPLE, 1)).float()[0]
        cdf = self.dist.probs.cumsum(-1)
        H.t += 1
        return (u >= cdf[..., :-1]).sum(-1).long()

    class Loader:
        def __init__(self, dataset, batch_size, shuffle):
            self.ds, self.bs, self.epoch = dataset, batch_size, 0

        def __iter__(self):
            perm = epoch_permutation(H.seed, H.update, self.epoch, len(self.ds))
            H.epoch = self.epoch
            self.epoch += 1
            for k in range(0, len(self.ds), self.bs):
                H.mb = k // self.bs
                yield self.ds[perm[k:k + self.bs]]

    class CoinDropout(torch.nn.Module):
        def forward(self, x):
            if not self.training:
                return x
            return x * float(reward_coin(H.seed, H.update, H.epoch, H.mb, H.p_reward))

    X.Discrete.sample = icdf_sample
    X.DataLoader = Loader
    wm = dict(attn_dim_head=16, heads=4, depth=depth)
    if gates:
        wm.update(attn_gate_values=True, add_value_residual=True, learned_value_residual_mix=True)
    torch.manual_seed(seed)
    learner = X.Learner(state_dim=S, num_actions=A, reward_range=(-2., 2.), world_model=wm, max_timesteps=T,
                        batch_size=batch, num_episodes_per_update=episodes, evolutionary=evolutionary,
                        evolve_every=1, evolve_after_step=0,
                        latent_gene_pool=dict(dim=gene_dim, num_genes_per_island=3, num_selected=2, tournament_size=2),
                        agent_kwargs=dict(dropout=0.))
    agent = learner.agent
    agent.save_path = Path('/tmp/xtrl_golden_ppo.pt')
    agent.model.reward_dropout = CoinDropout()
    if evolutionary:
        orig_evolve = agent.gene_pool.evolve_

        def evolve_(fitnesses, *a, **k):
            torch.manual_seed(evolve_seed(H.seed, H.update, H.epoch, H.mb))
            return orig_evolve(fitnesses, *a, **k)
        agent.gene_pool.evolve_ = evolve_
    init_sd = {k: v.clone() for k, v in agent.model.state_dict().items()}
    init_genes = agent.gene_pool.genes.detach().clone() if evolutionary else torch.zeros(1)
    learner.accelerator.log = lambda logs, *a, **k: H.logs.append(
        {kk: float(vv.mean()) for kk, vv in logs.items()})
    orig_learn = agent.learn

    def learn(memories, episode_lens, gene_ids, fitnesses=None):
        H.learn_inputs.append((list(memories), episode_lens.clone(), gene_ids.clone(),
                               None if fitnesses is None else fitnesses.clone()))
        orig_learn(memories, episode_lens, gene_ids, fitnesses)
        H.update += 1
        H.slot = -1
    agent.learn = learn
    learner(Sim(), updates)

    out = dict(cfg=np.array([seed, S, A, T, depth, int(gates), int(evolutionary), episodes, batch, updates,
                             hazard_log2, gene_dim], dtype=np.int64),
               mode=np.array(mode), reward_dropout=np.float32(reward_dropout), init_genes=init_genes)
    out.update(sd_arrays('init.', init_sd))
    out.update(sd_arrays('final.', agent.model.state_dict()))
    out.update(sd_arrays('ema.', agent.ema_model.ema_model.state_dict()))
    out.update(rs_mean=agent.rsnorm.running_mean, rs_var=agent.rsnorm.running_variance, rs_step=agent.rsnorm.step)
    if evolutionary:
        out.update(final_genes=agent.gene_pool.genes.detach())
    for u, (mems, lens, genes, fit) in enumerate(H.learn_inputs):
        cols = list(zip(*[tuple(map(torch.stack, zip(*ep))) for ep in mems]))
        names = ('states', 'actions', 'logp', 'rewards', 'bounds', 'values')
        for nm, col in zip(names, cols):
            out[f'u{u}.{nm}'] = torch.nn.utils.rnn.pad_sequence(list(col), batch_first=True)
        out[f'u{u}.lens'] = lens
        out[f'u{u}.genes'] = genes
        if fit is not None:
            out[f'u{u}.fitness'] = fit
    keys = list(H.logs[0].keys())
    out['log_keys'] = np.array(keys)
    out['logs'] = np.array([[lg.get(k, np.nan) for k in keys] for lg in H.logs], dtype=np.float64)
    save(name, **out)


def main():
    mods = load_reference()
    X, E = mods['x_transformers_rl'], mods['evolution']
    gen_fractal(mods['fractal_rl'])
    if sys.argv[1:] == ['fractal']:     # only the fractal fixtures
        return
    gen_gae(X)
    gen_rsnorm(X)
    gen_normalize_and_dists(X)
    gen_losses(X)
    gen_model_forward(X)
    gen_evolve(X, E)
    gen_learner(X, 'learner_readme', seed=7, S=5, A=2, T=10, depth=1, gates=False, evolutionary=False, episodes=4,
                batch=2, updates=2, mode='readme', hazard_log2=0, reward_dropout=0.5)
    gen_learner(X, 'learner_lander_evo', seed=11, S=8, A=4, T=24, depth=2, gates=True, evolutionary=True,
                episodes=4, batch=4, updates=2, mode='lander', hazard_log2=3, reward_dropout=0.5)


if __name__ == '__main__':
    main()
