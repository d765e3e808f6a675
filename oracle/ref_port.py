"""CPU restatement of the reference Learner hot path — TEST INFRASTRUCTURE ONLY (see oracle/__init__).

Every function cites the reference line it restates (``xtrl.py`` = x_transformers_rl/x_transformers_rl.py,
``evo.py`` = x_transformers_rl/evolution.py of the 2025-07-04 snapshot).  Pinned by the golden
vectors in tests/golden/ (produced by running those very lines in this container); the
third-party pieces come from oracle/thirdparty.py and are parity-unpinned.

Sampling protocol: torch.multinomial's CPU stream cannot be reproduced on a GPU, so
both this oracle and the HIP path sample a categorical by inverse CDF on a supplied uniform u:
    action = #{ i < A-1 : u >= cumsum(p)[i] }      (p = Categorical-normalised softmax)
which is the distribution torch draws from; the uniforms come from oracle/philox.py.
"""
from __future__ import annotations

import math
from copy import deepcopy
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn
from torch.nn.utils.rnn import pad_sequence

from . import thirdparty as tp
from .philox import (FIELD_COIN, FIELD_SAMPLE, SynthSim, attn_dropout_keep, epoch_permutation, evolve_seed,
                     ff_dropout_keep, philox_uniform, reward_coin)

F32_EPS = float(torch.finfo(torch.float32).eps)

# --------------------------------------------------------------------------------------------
# helpers  (xtrl.py:103-177)
# --------------------------------------------------------------------------------------------


def normalize(t, mask=None, eps=1e-5):
    """xtrl.py:103-112 — standardise with mean / unbiased var over the masked entries."""
    sel = t[mask] if mask is not None else t
    if sel.numel() == 0:
        return t
    return (t - sel.mean()) / sel.var().clamp(min=eps).sqrt()


def frac_gradient(t, frac):
    """xtrl.py:114-116 — identity forward, gradient scaled by ``frac``."""
    return t.detach() * (1. - frac) + t * frac


def shift_right(t, fill):
    """xtrl.py:911-918 — F.pad(t, (1, -1)) along time (dim 1)."""
    out = torch.full_like(t, fill)
    out[:, 1:] = t[:, :-1]
    return out


# --------------------------------------------------------------------------------------------
# distributions  (xtrl.py:181-277; torch.distributions semantics)
# --------------------------------------------------------------------------------------------


def safe_embed(weight, actions):
    """xtrl.py:181-195 — negative action id -> zero vector."""
    has = actions >= 0
    emb = weight[torch.where(has, actions, torch.zeros_like(actions))]
    return emb * has[..., None].to(emb.dtype)


def categorical_logits(raw):
    """xtrl.py:203-204 softmax, then torch Categorical(probs): p/sum(p), logits = log(clamp(p, eps, 1-eps))."""
    probs = raw.softmax(dim=-1)
    probs = probs / probs.sum(-1, keepdim=True)
    return probs, probs.clamp(F32_EPS, 1. - F32_EPS).log()


def discrete_log_prob(raw, actions):
    _, logits = categorical_logits(raw)
    return logits.gather(-1, actions.long()[..., None])[..., 0]


def discrete_entropy(raw):
    probs, logits = categorical_logits(raw)
    return -(logits.clamp(min=torch.finfo(logits.dtype).min) * probs).sum(-1)


def discrete_sample_icdf(raw, u):
    """Inverse-CDF sample on supplied uniforms (the shared-uniform protocol, module docstring)."""
    probs, _ = categorical_logits(raw)
    cdf = probs.cumsum(-1)
    return (u[..., None] >= cdf[..., :-1]).sum(-1).long()


def continuous_params(raw):
    """xtrl.py:232-244 — interleaved (mean, logvar); var = exp(3 tanh(lv/3))."""
    r = raw.reshape(*raw.shape[:-1], -1, 2)
    mean, lv = r.unbind(-1)
    var = (torch.tanh(lv / 3.) * 3.).exp()
    return mean, var


def continuous_log_prob(raw, value, squash):
    """xtrl.py:265-271 with torch Normal(mean, sqrt(clamp(var, 1e-5)))."""
    mean, var = continuous_params(raw)
    std = var.clamp(min=1e-5).sqrt()
    lp = -((value - mean) ** 2) / (2 * std ** 2) - std.log() - math.log(math.sqrt(2 * math.pi))
    if squash:
        lp = lp - (1. - value.pow(2)).clamp(min=1e-20).log()
    return lp


def continuous_entropy(raw):
    mean, var = continuous_params(raw)
    std = var.clamp(min=1e-5).sqrt()
    return 0.5 + 0.5 * math.log(2 * math.pi) + std.log()


def continuous_sample(raw, z, squash):
    """Reparameterised sample with supplied standard normals z (shared-uniform protocol)."""
    mean, var = continuous_params(raw)
    s = mean + var.clamp(min=1e-5).sqrt() * z
    return s.tanh() if squash else s


# --------------------------------------------------------------------------------------------
# RSNorm  (xtrl.py:565-612)
# --------------------------------------------------------------------------------------------


@dataclass
class RSNormState:
    dim: int
    eps: float = 1e-5
    step: int = 1
    mean: torch.Tensor = None
    var: torch.Tensor = None

    def __post_init__(self):
        if self.mean is None:
            self.mean = torch.zeros(self.dim)
        if self.var is None:
            self.var = torch.ones(self.dim)

    def apply(self, x):
        """xtrl.py:591 — (x - mean) / clamp(sqrt(var), eps)."""
        return (x - self.mean) / self.var.sqrt().clamp(min=self.eps)

    def train_call(self, x, allreduce_mean=None):
        """xtrl.py:586-612 — output uses OLD stats; then mean-of-batch update of the stats."""
        out = self.apply(x)
        m = x.reshape(-1, self.dim).mean(0)
        if allreduce_mean is not None:
            m = allreduce_mean(m)
        t = self.step
        delta = m - self.mean
        new_mean = self.mean + delta / t
        new_var = (t - 1) / t * (self.var + delta ** 2 / t)
        self.mean, self.var, self.step = new_mean, new_var, t + 1
        return out

    def copy(self):
        return RSNormState(self.dim, self.eps, self.step, self.mean.clone(), self.var.clone())


# --------------------------------------------------------------------------------------------
# GAE  (xtrl.py:616-640) — sequential reverse scan (the canonical order the HIP kernel follows)
# --------------------------------------------------------------------------------------------


def calc_gae(rewards, values, masks, gamma=0.99, lam=0.95, boot=None, lens=None):
    """xtrl.py:616-640.  ``boot`` [b] (NaN: none) with ``lens``: the value of the state after a
    truncated episode's last step (the bootstrap memory of xtrl.py:1323-1336) stands in for v at
    index lens[i] — what the reference's GAE would read had that memory joined its episode."""
    v = F.pad(values, (0, 1), value=0.)
    if boot is not None:
        v = v.clone()
        for i, (bv, le) in enumerate(zip(boot.tolist(), lens.tolist())):
            if bv == bv:
                v[i, le] = bv
    v_now, v_next = v[..., :-1], v[..., 1:]
    delta = rewards + gamma * v_next * masks - v_now
    gates = gamma * lam * masks
    gae = torch.empty_like(delta)
    acc = torch.zeros_like(delta[..., 0])
    for t in range(delta.shape[-1] - 1, -1, -1):
        acc = gates[..., t] * acc + delta[..., t]
        gae[..., t] = acc
    return gae + v_now


# --------------------------------------------------------------------------------------------
# WorldModelActorCritic  (xtrl.py:281-559) — reference parameter names
# --------------------------------------------------------------------------------------------


@dataclass
class ModelConfig:
    state_dim: int
    num_actions: int
    dim: int = 48
    depth: int = 1
    heads: int = 4
    dim_head: int = 16
    max_timesteps: int = 500
    reward_range: tuple = (-1., 1.)
    num_bins: int = 100
    continuous: bool = False
    squash: bool = True
    evolutionary: bool = False
    dim_gene: int = 0
    frac_head_grad: float = 0.5
    entropy_weight: float = 0.01
    eps_clip: float = 0.2
    value_clip: float = 0.4
    dropout: float = 0.
    reward_dropout: float = 0.5
    normalize_advantages: bool = True
    # world_model dict flags splatted into Decoder (xtrl.py:726-733; README uses none of them,
    # train_lander.py:43-50 turns all three on)
    gate_values: bool = False
    value_residual: bool = False
    learned_mix: bool = False
    ff_mult: int = 4          # x-transformers FeedForward mult, reached through world_model['ff_mult']
    ff_no_bias: bool = False  # world_model['ff_no_bias'] (x-transformers FeedForward no_bias)
    ff_glu: bool = False      # world_model['ff_glu'] (x-transformers FeedForward glu: GELU-gated project-in)
    rms_norm: bool = False    # world_model['use_rmsnorm'] (x-transformers RMSNorm pre-norms / final norm)
    qk_norm: bool = False     # world_model['attn_qk_norm'] (+ attn_qk_norm_scale)
    qk_norm_scale: float = 10.
    rotary_xpos: bool = False  # world_model['rotary_xpos'] (+ rotary_xpos_scale_base)
    xpos_scale_base: float = 512.


class OracleWMAC(nn.Module):
    """Restatement of WorldModelActorCritic (xtrl.py:281-392 layout, 479-559 forward)."""

    def __init__(self, cfg: ModelConfig):
        super().__init__()
        d = cfg.dim
        self.cfg = cfg
        self.transformer = tp.ContinuousTransformerWrapper(
            dim_in=cfg.state_dim, dim_out=None, max_seq_len=cfg.max_timesteps, probabilistic=True,
            attn_layers=tp.Decoder(dim=d, depth=cfg.depth, heads=cfg.heads, attn_dim_head=cfg.dim_head,
                                   rotary_pos_emb=True, attn_dropout=cfg.dropout, ff_dropout=cfg.dropout,
                                   verbose=False, attn_gate_values=cfg.gate_values,
                                   add_value_residual=cfg.value_residual,
                                   learned_value_residual_mix=cfg.learned_mix, ff_mult=cfg.ff_mult,
                                   ff_no_bias=cfg.ff_no_bias, ff_glu=cfg.ff_glu, attn_qk_norm=cfg.qk_norm,
                                   attn_qk_norm_scale=cfg.qk_norm_scale, rotary_xpos=cfg.rotary_xpos,
                                   rotary_xpos_scale_base=cfg.xpos_scale_base, use_rmsnorm=cfg.rms_norm))
        self.reward_embed = nn.Parameter(torch.ones(d) * 1e-2)
        if cfg.continuous:
            self.action_embeds = nn.Linear(cfg.num_actions, d)
        else:
            self.action_embeds = nn.Module()
            self.action_embeds.embed = nn.Embedding(cfg.num_actions, d)
        self.to_state_embed = nn.Linear(cfg.state_dim, d)
        self.to_pred_done = nn.Sequential(nn.Linear(2 * d, 1))
        self.to_pred = nn.Sequential(nn.Linear(2 * d, d), nn.SiLU(), nn.Linear(d, 2 * (cfg.state_dim + 1)))
        in_dim = 2 * d
        if cfg.evolutionary:
            self.latent_to_embed = nn.Linear(cfg.dim_gene, d)
            in_dim += d
        n_out = cfg.num_actions * (2 if cfg.continuous else 1)
        self.critic_head = nn.Sequential(nn.Linear(in_dim, 2 * d), nn.SiLU(), nn.Linear(2 * d, cfg.num_bins))
        self.action_head = nn.Sequential(nn.Linear(in_dim, 2 * d), nn.SiLU(), nn.Linear(2 * d, n_out))
        self.hl = tp.HLGaussLoss(cfg.reward_range[0], cfg.reward_range[1], cfg.num_bins, clamp_to_range=True)

    def embed_actions(self, actions):
        if self.cfg.continuous:
            return self.action_embeds(actions)
        return safe_embed(self.action_embeds.embed.weight, actions)

    def forward(self, state, actions=None, rewards=None, next_actions=None, latent_gene=None,
                mask=None, cache=None, reward_keep=True):
        """xtrl.py:479-559.  ``reward_keep`` is the all-or-nothing reward-dropout coin (:501-503)."""
        state_embed = self.to_state_embed(state)
        sum_embeds = 0.
        if actions is not None:
            sum_embeds = sum_embeds + self.embed_actions(actions)
        if rewards is not None:
            sum_embeds = sum_embeds + rewards[..., None] * self.reward_embed * float(reward_keep)
        embed, new_cache = self.transformer(state, mask=mask, cache=cache, sum_embeds=sum_embeds,
                                            return_embeddings=True, return_intermediates=True)
        state_pred = dones = None
        if next_actions is not None:
            ewa = torch.cat((embed, self.embed_actions(next_actions)), dim=-1)
            mean, var = continuous_params(self.to_pred(ewa))
            state_pred = torch.stack((mean, var))
            dones = self.to_pred_done(ewa)[..., 0].sigmoid()
        embed = frac_gradient(embed, self.cfg.frac_head_grad)
        ac_in = torch.cat((embed, state_embed), dim=-1)
        if self.cfg.evolutionary:
            lat = self.latent_to_embed(latent_gene)
            if lat.ndim == 2:
                lat = lat[:, None, :].expand(-1, ac_in.shape[1], -1)
            ac_in = torch.cat((ac_in, lat), dim=-1)
        return self.action_head(ac_in), self.critic_head(ac_in), state_pred, dones, new_cache


# --------------------------------------------------------------------------------------------
# losses  (xtrl.py:398-477, 939-978)
# --------------------------------------------------------------------------------------------


def autoregressive_loss(state_pred, real):
    """xtrl.py:398-404 — F.gaussian_nll_loss(mean[:, :-1], real[:, 1:], var[:, :-1], 'none')."""
    mean, var = state_pred[0][:, :-1], state_pred[1][:, :-1]
    return F.gaussian_nll_loss(mean, real[:, 1:], var, reduction='none')


def done_loss(done_pred, dones):
    """xtrl.py:406-411."""
    return F.binary_cross_entropy(done_pred, dones.to(done_pred.dtype), reduction='none')


def actor_loss(cfg, hl, raw, actions, old_log_probs, returns, old_values, mask):
    """xtrl.py:413-444."""
    if cfg.continuous:
        lp = continuous_log_prob(raw, actions, cfg.squash)
        ent = -lp if cfg.squash else continuous_entropy(raw)
    else:
        lp = discrete_log_prob(raw, actions)
        ent = discrete_entropy(raw)
    ratios = (lp - old_log_probs).exp()
    clipped = ratios.clamp(1 - cfg.eps_clip, 1 + cfg.eps_clip)
    adv = returns - hl(old_values).detach()
    if cfg.normalize_advantages:
        adv = normalize(adv, mask)
    extra = ratios.ndim - adv.ndim
    adv = adv.reshape(*adv.shape, *((1,) * extra))
    loss = -torch.min(ratios * adv, clipped * adv) - cfg.entropy_weight * ent
    return loss.reshape(*loss.shape[:2], -1).sum(-1)


def critic_loss(cfg, hl, values, returns, old_values):
    """xtrl.py:446-477."""
    clip = cfg.value_clip
    v_old, v = hl(old_values), hl(values)
    clipped_loss = hl(values, returns.clamp(-clip, clip))
    loss = hl(values, returns)
    lo, hi = v_old - clip, v_old + clip
    between = lambda mid, a, b: (a < mid) & (mid < b)
    return torch.where(between(v, returns, lo) | between(v, hi, returns), 0., torch.min(loss, clipped_loss))


@dataclass
class Minibatch:
    states: torch.Tensor        # (b, n, S)
    actions: torch.Tensor       # (b, n) long | (b, n, A)
    rewards: torch.Tensor       # (b, n)
    old_log_probs: torch.Tensor  # (b, n) | (b, n, A)
    returns: torch.Tensor       # (b, n)
    old_values: torch.Tensor    # (b, n, B)
    dones: torch.Tensor         # (b, n) bool
    gene_ids: torch.Tensor      # (b,)
    episode_lens: torch.Tensor  # (b,)


@dataclass
class LossWeights:
    actor: float = 1.
    critic: float = 1.
    autoregressive: float = 1.


def minibatch_loss(model: OracleWMAC, rsnorm: RSNormState, mb: Minibatch, latent_gene=None,
                   weights: LossWeights = LossWeights(), reward_keep=True):
    """xtrl.py:903-978 — returns (loss, logs, normalised states_with_rewards, mask)."""
    cfg = model.cfg
    n = mb.states.shape[1]
    mask = torch.arange(n)[None, :] < mb.episode_lens[:, None]
    prev_actions = shift_right(mb.actions, 0. if cfg.continuous else -1)
    rewards = shift_right(mb.rewards, 0.)
    swr = torch.cat((mb.states, rewards[..., None]), dim=-1)
    with torch.no_grad():
        swr = rsnorm.apply(swr)
    states, rewards = swr[..., :-1], swr[..., -1]
    raw, values, pred, done_pred, _ = model(states, actions=prev_actions, rewards=rewards,
                                            next_actions=mb.actions, latent_gene=latent_gene,
                                            mask=mask, reward_keep=reward_keep)
    wm = autoregressive_loss(pred, swr)[mask[:, :-1]]
    dl = done_loss(done_pred, mb.dones)[mask]
    al = actor_loss(cfg, model.hl, raw, mb.actions, mb.old_log_probs, mb.returns, mb.old_values, mask)
    cl = critic_loss(cfg, model.hl, values, mb.returns, mb.old_values)
    ac = (al * weights.actor + cl * weights.critic)[mask]
    loss = ac.mean() + (wm.mean() + dl.mean()) * weights.autoregressive
    logs = dict(actor_loss=al.mean(), critic_loss=cl.mean(), autoreg_loss=wm.mean(), pred_done_loss=dl.mean())
    return loss, logs, swr, mask


class PhiloxAttnDropout(nn.Module):
    """x-transformers' attention-probability dropout (xtrl.py:729 attn_dropout) with the keep mask of
    the shared counter-based stream (philox.attn_dropout_keep) in place of torch's RNG: the same
    probabilities are dropped as in the HIP training attention, so the two can be compared with
    dropout on.  Applies only in training mode, like nn.Dropout."""

    def __init__(self, layer, p=0., seed=0, offset=0):
        super().__init__()
        self.layer, self.p, self.seed, self.offset = layer, p, seed, offset

    def forward(self, attn):
        if not self.training or self.p <= 0.:
            return attn
        b, h, n, j = attn.shape
        assert n == j, 'training attention (no cache)'
        keep = torch.from_numpy(attn_dropout_keep(b, h, n, self.p, self.seed, self.offset, self.layer))
        return attn * keep.to(attn.dtype) / (1. - self.p)


class PhiloxFFDropout(nn.Module):
    """FeedForward's Dropout after GELU (xtrl.py:730 ff_dropout) with philox.ff_dropout_keep over the
    minibatch's token-major rows (episode * n + step) — the GPU's GELU + dropout GEMM epilogue mask."""

    def __init__(self, layer, p=0., seed=0, offset=0):
        super().__init__()
        self.layer, self.p, self.seed, self.offset = layer, p, seed, offset
        self.packed_lens = None

    def forward(self, h):
        if not self.training or self.p <= 0.:
            return h
        b, n, f = h.shape
        if self.packed_lens is None:
            keep = torch.from_numpy(ff_dropout_keep(b * n, f, self.p, self.seed, self.offset, self.layer))
        else:   # the packed learn step (XtrlTrainDesc.packed): rows numbered over the valid tokens only,
            # episode after episode; the padded tokens' mask is irrelevant (no loss term reaches them)
            ln = np.minimum(np.asarray(self.packed_lens, dtype=np.int64), n)
            kp = ff_dropout_keep(int(ln.sum()), f, self.p, self.seed, self.offset, self.layer)
            keep = np.ones((b * n, f), dtype=kp.dtype)
            rows = np.concatenate([e * n + np.arange(ln[e]) for e in range(b)]) if b else np.zeros(0, np.int64)
            keep[rows] = kp
            keep = torch.from_numpy(keep)
        return h * keep.reshape(b, n, f).to(h.dtype) / (1. - self.p)


def install_philox_dropout(model, p, seed, attn_offset, ff_offset, packed_lens=None):
    """Point every attention / feed-forward dropout of an OracleWMAC decoder at the learn step's
    counter-based streams for one minibatch (seed = agent seed * 1000003 + update, attention counters
    from ``attn_offset``, FF counter ``ff_offset``; the layer index in the Philox sub-index, as
    xtrl_amd.learner.Agent.learn draws them)."""
    layers = model.transformer.attn_layers.layers
    for li in range(len(layers) // 2):
        attn, ff = layers[2 * li][1], layers[2 * li + 1][1]
        if not isinstance(attn.attn_dropout, PhiloxAttnDropout):
            attn.attn_dropout = PhiloxAttnDropout(li)
            ff.ff[1] = PhiloxFFDropout(li)
        for m, off in ((attn.attn_dropout, attn_offset), (ff.ff[1], ff_offset)):
            m.p, m.seed, m.offset = float(p), int(seed), int(off)
            m.train(model.training)
        ff.ff[1].packed_lens = None if packed_lens is None else [int(x) for x in packed_lens]


# --------------------------------------------------------------------------------------------
# LatentGenePool.evolve_  (evo.py:28-184) — same torch RNG call order as the reference
# --------------------------------------------------------------------------------------------


def l2norm(t):
    return F.normalize(t, dim=-1)


@torch.no_grad()
def evolve(genes, fitnesses, num_islands, num_selected, tournament_size, num_elites=1,
           mutation_std=0.1, migrate_every=10, frac_migrate=0.1, step=0, temperature=1.5):
    """evo.py:76-184 for the raw (un-normalised) gene parameter; returns new raw genes."""
    G, D = genes.shape
    per = G // num_islands
    n_children = per - num_selected
    fit = fitnesses.reshape(num_islands, per)
    g = genes.reshape(num_islands, per, D)
    sorted_fit, sorted_ids = fit.sort(dim=-1, descending=True)
    sel_ids = sorted_ids[:, :num_selected]
    selected = g.gather(1, sel_ids[..., None].expand(-1, -1, D))
    tourn = torch.randn((num_islands, n_children, num_selected)).argsort(dim=-1)[..., :tournament_size]
    # evo.py:117-119 gathers the *sorted* fitness by tournament ids along dim 1
    sf = sorted_fit[..., None].expand(-1, -1, tourn.shape[-1])
    tourn_fit = sf.gather(1, tourn)
    parent_ids = tourn_fit.topk(2, dim=-1).indices.reshape(num_islands, -1)
    parents = selected.gather(1, parent_ids[..., None].expand(-1, -1, D))
    parents = parents.reshape(num_islands, n_children, 2, D).permute(2, 0, 1, 3)
    p1, p2 = parents[0], parents[1]
    children = p1.lerp(p2, (torch.randn_like(p1) / temperature).sigmoid())
    if (step + 1) % migrate_every == 0 and num_islands > 1 and frac_migrate > 0.:
        if num_elites > 0:
            elites, selected = selected[:, :1], selected[:, 1:]
        k = max(1, int(selected.shape[1] * frac_migrate))
        selected, migrants = selected[:, -k:], selected[:, :-k]
        selected = torch.cat((selected, torch.roll(migrants, 1, dims=(1,))), dim=1)
        if num_elites > 0:
            selected = torch.cat((elites, selected), dim=1)
    out = torch.cat((selected, children), dim=1)
    if mutation_std > 0:
        if num_elites > 0:
            el, rest = out[:, :1], out[:, 1:]
        else:
            el, rest = None, out
        rest = rest + torch.randn_like(rest) * mutation_std
        out = torch.cat((el, rest), dim=1) if el is not None else rest
    return l2norm(out.reshape(G, D)), sel_ids


# --------------------------------------------------------------------------------------------
# Agent + Learner restated (xtrl.py:644-1380): batch-1 sequential rollout, the reference's learn
# --------------------------------------------------------------------------------------------


@dataclass
class LearnerConfig:
    state_dim: int
    num_actions: int
    reward_range: tuple
    dim: int = 48
    depth: int = 1
    heads: int = 4
    dim_head: int = 16
    gate_values: bool = False
    value_residual: bool = False
    learned_mix: bool = False
    ff_mult: int = 4
    ff_no_bias: bool = False
    ff_glu: bool = False
    rms_norm: bool = False
    qk_norm: bool = False
    qk_norm_scale: float = 10.
    rotary_xpos: bool = False
    xpos_scale_base: float = 512.
    continuous: bool = False
    squash: bool = True
    clamp: tuple | None = None
    sim_mode: str = 'readme'
    hazard_log2: int = 6
    evolutionary: bool = False
    evolve_every: int = 10
    evolve_after_step: int = 20
    gene_pool: dict = field(default_factory=lambda: dict(dim=128, num_genes_per_island=3, num_selected=2,
                                                         tournament_size=2))
    max_timesteps: int = 500
    batch_size: int = 8
    num_episodes_per_update: int = 64
    lr: float = 8e-4
    betas: tuple = (0.9, 0.99)
    lam: float = 0.95
    gamma: float = 0.99
    eps_clip: float = 0.2
    value_clip: float = 0.4
    beta_s: float = 0.01
    regen_reg_rate: float = 1e-4
    cautious_factor: float = 0.1
    epochs: int = 4
    ema_decay: float = 0.9
    frac_head_grad: float = 0.5
    dropout: float = 0.
    reward_dropout: float = 0.5
    max_grad_norm: float = 0.5
    weights: LossWeights = field(default_factory=LossWeights)
    seed: int = 0


class OracleLearner:
    """Batch-1 sequential Learner (xtrl.py:1174-1380 + Agent.learn :808-1023), with the
    shared-uniform sampling protocol and counter-based minibatch permutations / reward coins
    (oracle/philox.py) so that a vectorised GPU run can be compared step by step."""

    def __init__(self, c: LearnerConfig, init_state_dict=None, genes=None, model_factory=None):
        """``model_factory(ModelConfig) -> module`` swaps the policy body (OracleWMAC by default;
        fractal_ref.OracleFractalPolicy for the causal fractal body)."""
        self.c = c
        torch.manual_seed(c.seed)
        self.gp = None
        if c.evolutionary:
            gpc = dict(c.gene_pool)
            self.gp = dict(num_islands=gpc.pop('num_islands', 1), **gpc)
            n_genes = gpc['num_genes_per_island'] * self.gp['num_islands']
            self.genes = l2norm(torch.randn(n_genes, gpc['dim'])) if genes is None else genes.clone()
            self.gp_step = 0
        mc = ModelConfig(c.state_dim, c.num_actions, c.dim, c.depth, c.heads, c.dim_head, c.max_timesteps,
                         c.reward_range, 100, c.continuous, c.squash, c.evolutionary,
                         self.gp['dim'] if c.evolutionary else 0, c.frac_head_grad, c.beta_s, c.eps_clip,
                         c.value_clip, c.dropout, c.reward_dropout, True, c.gate_values, c.value_residual,
                         c.learned_mix, c.ff_mult, c.ff_no_bias, c.ff_glu, rms_norm=c.rms_norm, qk_norm=c.qk_norm,
                         qk_norm_scale=c.qk_norm_scale, rotary_xpos=c.rotary_xpos, xpos_scale_base=c.xpos_scale_base)
        self.model = model_factory(mc) if model_factory is not None else OracleWMAC(mc)
        if init_state_dict is not None:
            self.model.load_state_dict(init_state_dict)
        self.rsnorm = RSNormState(c.state_dim + 1)
        self.ema = tp.EMA(self.model, beta=c.ema_decay, include_online_model=False,
                          update_model_with_ema_every=1250)
        self.opt = tp.AdoptAtan2(self.model.parameters(), lr=c.lr, betas=c.betas,
                                 regen_reg_rate=c.regen_reg_rate, cautious_factor=c.cautious_factor)
        self.ema.add_to_optimizer_post_step_hook(self.opt)
        self.step = 0
        n_genes = self.genes.shape[0] if c.evolutionary else 1
        self.episode_genes = [(e, g) for e in range(c.num_episodes_per_update) for g in range(n_genes)]
        self.logs = []

    def latent(self, gene_ids):
        return l2norm(self.genes[gene_ids])

    @torch.no_grad()
    def rollout(self, update, max_timesteps=None, sim_seed=None, slots=None):
        """xtrl.py:1204-1356 for one learning update; env slot i = i-th (episode, gene) pair.
        ``slots``: replay only these pairs (a sample of a wide rollout; episodes come back in that order)."""
        c = self.c
        T = max_timesteps or c.max_timesteps
        model = self.ema.ema_model
        model.eval()
        episodes = []
        fitness = torch.zeros(len(self.genes) if c.evolutionary else 1)
        pairs = list(enumerate(self.episode_genes))
        if slots is not None:
            pairs = [pairs[int(s)] for s in slots]
        for slot, (episode, gene) in pairs:
            sim = SynthSim(sim_seed if sim_seed is not None else c.seed, update, episode, c.state_dim,
                           c.num_actions, c.sim_mode, c.hazard_log2)
            state = torch.from_numpy(sim.reset()).float()
            prev_action = torch.zeros(c.num_actions) if c.continuous else torch.tensor(-1)
            prev_reward = torch.tensor(0.)
            latent = self.latent(torch.tensor([gene])) if c.evolutionary else None
            cache = None
            mem = []
            total = 0.
            for t in range(T):
                swr = self.rsnorm.apply(torch.cat((state, prev_reward[None])))
                raw, values, _, _, cache = model(swr[:-1].reshape(1, 1, -1), actions=prev_action.reshape(1, 1, *prev_action.shape),
                                                 rewards=swr[-1], latent_gene=latent, cache=cache)
                raw, values = raw.reshape(-1), values.reshape(-1)
                u = torch.from_numpy(philox_uniform(c.seed, update, slot, t, FIELD_SAMPLE, 1)).float()
                if c.continuous:
                    z = torch.from_numpy(philox_uniform(c.seed, update, slot, t, FIELD_SAMPLE, c.num_actions,
                                                        normal=True)).float()
                    action = continuous_sample(raw, z, c.squash)
                    lp = continuous_log_prob(raw, action, c.squash)
                    if c.clamp is not None:
                        action = action.clamp(*c.clamp)
                else:
                    action = discrete_sample_icdf(raw, u[0])
                    lp = discrete_log_prob(raw, action)
                nxt, reward, terminated = sim.step(action.numpy())
                total += float(reward)
                mem.append((state, action, lp, torch.tensor(float(reward)), torch.tensor(bool(terminated)), values))
                prev_action, prev_reward = action, torch.tensor(float(reward))
                state = torch.from_numpy(nxt).float()
                if terminated:
                    break
            if c.evolutionary:
                fitness[gene] += total
            episodes.append(dict(mem=mem, len=t + 1, gene=gene))
        return episodes, fitness

    def rollout_env(self, env, update, max_timesteps=None, episode_seeds=None, bootstrap=True):
        """The reference loop against a host env (xtrl.py:1220-1341), batch 1, one env object for
        every (episode, gene) pair: reset(**{seed}) -> state | (state, ...); step(action.tolist())
        -> (s, r, terminated[, truncated, ...]) (a 4-tuple's 4th item is read as truncated,
        reference quirk B8); the memory stores is_boundary = terminated; done = terminated or
        truncated.  A truncated, not terminated episode gets the next state's value logits as
        ep['boot'] (xtrl.py:1323-1336) when ``bootstrap``."""
        c = self.c
        T = max_timesteps or c.max_timesteps
        model = self.ema.ema_model
        model.eval()
        episodes = []
        fitness = torch.zeros(len(self.genes) if c.evolutionary else 1)
        for slot, (episode, gene) in enumerate(self.episode_genes):
            kw = dict(seed=int(episode_seeds[episode])) if (c.evolutionary and episode_seeds is not None) else {}
            out = env.reset(**kw)
            state = torch.from_numpy(np.asarray(out[0] if isinstance(out, tuple) else out, dtype=np.float32))
            prev_action = torch.zeros(c.num_actions) if c.continuous else torch.tensor(-1)
            prev_reward = torch.tensor(0.)
            latent = self.latent(torch.tensor([gene])) if c.evolutionary else None
            cache = None
            mem, total, boot = [], 0., None

            def policy(state, prev_action, prev_reward, cache):
                swr = self.rsnorm.apply(torch.cat((state, prev_reward[None])))
                raw, values, _, _, cache = model(swr[:-1].reshape(1, 1, -1),
                                                 actions=prev_action.reshape(1, 1, *prev_action.shape),
                                                 rewards=swr[-1], latent_gene=latent, cache=cache)
                return raw.reshape(-1), values.reshape(-1), cache

            for t in range(T):
                raw, values, cache = policy(state, prev_action, prev_reward, cache)
                u = torch.from_numpy(philox_uniform(c.seed, update, slot, t, FIELD_SAMPLE, 1)).float()
                if c.continuous:
                    z = torch.from_numpy(philox_uniform(c.seed, update, slot, t, FIELD_SAMPLE, c.num_actions,
                                                        normal=True)).float()
                    action = continuous_sample(raw, z, c.squash)
                    lp = continuous_log_prob(raw, action, c.squash)
                    if c.clamp is not None:
                        action = action.clamp(*c.clamp)
                else:
                    action = discrete_sample_icdf(raw, u[0])
                    lp = discrete_log_prob(raw, action)
                o = env.step(action.tolist())
                if len(o) >= 4:
                    nxt, reward, terminated, truncated = o[:4]
                elif len(o) == 3:
                    (nxt, reward, terminated), truncated = o, False
                else:
                    raise RuntimeError('invalid number of returns from environment .step')
                reward = float(np.asarray(reward).reshape(-1)[0])
                total += reward
                prev_action, prev_reward = action, torch.tensor(reward)
                mem.append((state, action, lp, torch.tensor(reward), torch.tensor(bool(terminated)), values))
                state = torch.from_numpy(np.asarray(nxt, dtype=np.float32))
                done = bool(terminated) or bool(truncated)
                if done and not terminated and bootstrap:
                    _, boot, _ = policy(state, prev_action, prev_reward, cache)
                if done:
                    break
            if c.evolutionary:
                fitness[gene] += total
            episodes.append(dict(mem=mem, len=t + 1, gene=gene, boot=boot))
        return episodes, fitness

    def learn(self, episodes, fitness, update):
        """xtrl.py:808-1023."""
        c = self.c
        hl = self.model.hl
        cols = list(zip(*[tuple(map(torch.stack, zip(*ep['mem']))) for ep in episodes]))
        states, actions, old_lp, rewards, bounds, values = (pad_sequence(list(col), batch_first=True) for col in cols)
        lens = torch.tensor([ep['len'] for ep in episodes])
        gene_ids = torch.tensor([ep['gene'] for ep in episodes])
        boot = None
        if any(ep.get('boot') is not None for ep in episodes):
            boot = torch.tensor([float(hl(ep['boot'][None])[0]) if ep.get('boot') is not None else float('nan')
                                 for ep in episodes])
        returns = calc_gae(rewards, hl(values), (~bounds).float(), c.gamma, c.lam, boot, lens)
        rs_copy = self.rsnorm.copy()
        self.model.train()
        N = states.shape[0]
        for epoch in range(c.epochs):
            perm = epoch_permutation(c.seed, update, epoch, N)
            for mbi in range(0, N, c.batch_size):
                idx = perm[mbi:mbi + c.batch_size]
                mb = Minibatch(states[idx], actions[idx], rewards[idx], old_lp[idx], returns[idx], values[idx],
                               bounds[idx], gene_ids[idx], lens[idx])
                latent = self.latent(mb.gene_ids) if c.evolutionary else None
                keep = reward_coin(c.seed, update, epoch, mbi // c.batch_size, c.reward_dropout)
                loss, logs, swr, mask = minibatch_loss(self.model, self.rsnorm, mb, latent, c.weights, keep)
                loss.backward()
                nn.utils.clip_grad_norm_(self.model.parameters(), c.max_grad_norm)
                self.opt.step()
                self.opt.zero_grad()
                rs_copy.train_call(swr[mask])
                if c.evolutionary and self.step > c.evolve_after_step and self.step % c.evolve_every == 0:
                    gp = self.gp
                    torch.manual_seed(evolve_seed(c.seed, update, epoch, mbi // c.batch_size))
                    self.genes, _ = evolve(self.genes, fitness, gp['num_islands'], gp['num_selected'],
                                           gp['tournament_size'], step=self.gp_step)
                    self.gp_step += 1
                self.logs.append({k: float(v.detach()) for k, v in logs.items()} | dict(loss=float(loss.detach())))
        self.rsnorm = rs_copy
        self.step += 1

    def __call__(self, num_updates, max_timesteps=None):
        for u in range(num_updates):
            episodes, fitness = self.rollout(u, max_timesteps)
            self.learn(episodes, fitness, u)
