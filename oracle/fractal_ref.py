"""CPU restatement of the fractal policy body (TEST INFRASTRUCTURE: imported only by tests/).

Follows x_transformers_rl/fractal_rl.py in eval mode (dropout off), on a state_dict with the
reference's parameter names:
  FractalLevelEmbedding.forward            fractal_rl.py:64-68   (learned + sinusoidal scale, :50-62)
  FractalProcessingBlock.forward           fractal_rl.py:120-136 (post-norm: LN(x + attn(x)),
                                                                  LN(x + cross_attn(x, global)), LN(x + ff(x)))
  FractalEncoder.forward                   fractal_rl.py:274-346
  FractalWorldModelActorCritic.forward     fractal_rl.py:549-619
x-transformers Attention / FeedForward are not in the container; their semantics are
restated here: q, k, v, out projections without bias, heads split as (h, dh), scores q.k / sqrt(dh),
key-padding mask by -finfo.max, softmax, merge heads; FeedForward = Linear + GELU(erf) + Linear.
The parameter layout these imply is pinned by the parameter-count KATs of comprehensive_demo.py
(:338-357) and by the key set of the committed fractal_experiments/frala_easy_final checkpoint;
the numerics of the third-party modules are "parity unpinned" (no reference output exists).
The cross-attention here is computed in full (softmax over the one-token context) — the HIP path
uses its exact simplification (weights identically 1), so the test checks that too.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def param_count_encoder(input_dim, embed_dim, num_levels, heads, dim_head=64, ff_mult=4, share_weights=False,
                        use_hypernetwork=False, global_state_dim=None):
    """Parameter count of FractalEncoder (fractal_rl.py:140-235) under the restated layout."""
    d, g, inner = embed_dim, global_state_dim or embed_dim, heads * dim_head
    lin = lambda i, o, bias=True: i * o + (o if bias else 0)
    attn = 4 * d * inner                       # to_q, to_k, to_v (no bias), to_out (no bias)
    ff = lin(d, d * ff_mult) + lin(d * ff_mult, d)
    block = 2 * attn + ff + 3 * 2 * d          # self + global attention, ff, three affine LayerNorms
    n = lin(input_dim, d) + num_levels * d + g + lin(d, g)
    if share_weights:
        n += block
    elif use_hypernetwork:
        n += lin(d, 2 * d) + lin(2 * d, d) + block
    else:
        n += num_levels * block
    n += 2 * (num_levels - 1) * lin(d, d)      # upscale / downscale layers (built, unused in forward)
    n += num_levels * lin(d, d)                # level projections
    n += lin(d * (num_levels + 1), 2 * d) + lin(2 * d, d)
    return n


def _linear(x, sd, name, bias=True):
    w = sd[name + '.weight']
    b = sd.get(name + '.bias') if bias else None
    return F.linear(x, w, b)


def _attention(x, ctx, sd, pre, heads, dim_head, key_mask=None):
    """x-transformers Attention (no rotary, not causal): x [b, i, d], ctx [b, j, d]."""
    b, i, _ = x.shape
    j = ctx.shape[1]
    q = _linear(x, sd, pre + '.to_q', False).view(b, i, heads, dim_head).transpose(1, 2)
    k = _linear(ctx, sd, pre + '.to_k', False).view(b, j, heads, dim_head).transpose(1, 2)
    v = _linear(ctx, sd, pre + '.to_v', False).view(b, j, heads, dim_head).transpose(1, 2)
    sim = q @ k.transpose(-1, -2) / math.sqrt(dim_head)
    if key_mask is not None:
        sim = sim.masked_fill(~key_mask[:, None, None, :], -torch.finfo(sim.dtype).max)
    out = sim.softmax(dim=-1) @ v
    out = out.transpose(1, 2).reshape(b, i, heads * dim_head)
    return _linear(out, sd, pre + '.to_out', False)


def _layernorm(x, sd, name):
    return F.layer_norm(x, x.shape[-1:], sd[name + '.weight'], sd[name + '.bias'], eps=1e-5)


def _block(x, g, sd, pre, heads, dim_head, key_mask=None):
    """FractalProcessingBlock.forward (fractal_rl.py:120-136), use_global_attention=True; ``g`` None
    skips the global-state read and its norm (:126)."""
    x = _layernorm(x + _attention(x, x, sd, pre + '.self_attn', heads, dim_head, key_mask), sd, pre + '.norm1')
    if g is not None:
        x = _layernorm(x + _attention(x, g, sd, pre + '.global_attn', heads, dim_head), sd, pre + '.norm2')
    h = F.gelu(_linear(x, sd, pre + '.ff.ff.0.0'))
    return _layernorm(x + _linear(h, sd, pre + '.ff.ff.2'), sd, pre + '.norm3')


def encoder_forward(sd, x, num_levels, heads, dim_head, share_weights=False, use_hypernetwork=False, key_mask=None,
                    pre='fractal_encoder'):
    """FractalEncoder.forward (fractal_rl.py:274-346): returns (aggregated [b, d], level outputs)."""
    b = x.shape[0]
    k = (lambda name: f'{pre}.{name}') if pre else (lambda name: name)
    x = _linear(x, sd, k('input_embed'))
    g = sd[k('global_state_init')].expand(b, -1, -1)
    levels, cur = [], x
    for li in range(num_levels):
        emb = sd[k('level_embedding.level_embeds')][li] + sd[k('level_embedding.scale_embeds')][li]
        feats = cur + emb
        blk = k('fractal_block' if share_weights else 'base_block' if use_hypernetwork else f'fractal_blocks.{li}')
        feats = _block(feats, g, sd, blk, heads, dim_head, key_mask)
        g = g + _linear(feats.mean(dim=1, keepdim=True), sd, k('global_state_update'))
        levels.append(feats)
        cur = feats
    pooled = [_linear(lv, sd, k(f'level_projections.{i}')).mean(dim=1) for i, lv in enumerate(levels)]
    allf = torch.cat(pooled + [g.mean(dim=1)], dim=-1)
    agg = _linear(F.relu(_linear(allf, sd, k('final_aggregation.0'))), sd, k('final_aggregation.2'))
    return agg, levels


def world_model_forward(sd, state, num_levels, heads, dim_head, share_weights=False, use_hypernetwork=False,
                        next_actions=None, latent_gene=None, continuous=False, pre='world_model'):
    """FractalWorldModelActorCritic.forward (fractal_rl.py:549-619): (raw_actions, values, state_pred,
    dones, level outputs).  state [b, n, S]; next_actions [b] (discrete, -1 = none) or [b, A]."""
    s = {k[len(pre) + 1:]: v for k, v in sd.items() if k.startswith(pre + '.')} if pre else sd
    feats, levels = encoder_forward(s, state, num_levels, heads, dim_head, share_weights, use_hypernetwork)
    state_embed = _linear(state, s, 'to_state_embed')
    state_pred = dones = None
    if next_actions is not None:
        if continuous:
            na = _linear(next_actions, s, 'action_embeds')
        else:
            w = s['action_embeds.embed.weight']
            na = torch.where((next_actions >= 0)[:, None], w[next_actions.clamp(min=0)], torch.zeros_like(w[:1]))
        ewa = torch.cat((feats, na), dim=-1)
        raw = _linear(F.silu(_linear(ewa, s, 'to_pred.0')), s, 'to_pred.2')
        raw = raw.view(*raw.shape[:-1], -1, 2)
        mean, lv = raw.unbind(-1)
        state_pred = torch.stack((mean, (torch.tanh(lv / 3.) * 3.).exp()))
        dones = torch.sigmoid(_linear(ewa, s, 'to_pred_done.0')).squeeze(-1)
    if state_embed.ndim == 3:
        state_embed = state_embed.mean(dim=1)
    ac = torch.cat((feats, state_embed), dim=-1)
    if latent_gene is not None and 'latent_to_embed.weight' in s:
        ac = torch.cat((ac, _linear(latent_gene, s, 'latent_to_embed')), dim=-1)
    raw_actions = _linear(F.silu(_linear(ac, s, 'action_head.0')), s, 'action_head.2')
    values = _linear(F.silu(_linear(ac, s, 'critic_head.0')), s, 'critic_head.2')
    return raw_actions, values, state_pred, dones, levels


# ----------------------------------------------------------------------------------------------
# Per-timestep causal fractal policy body (xtrl_amd.fractal.FractalPolicyActorCritic) restated as
# the streaming loop a batch-1 rollout would run: position t sees states 0..t only.  Design (DESIGN
# §6, the reference never wires FractalWorldModelActorCritic into its Agent, fractal_rl.py:622-659):
#   per level l:  x <- x + level_emb_l;  x1 = LN1(x + SelfAttn(x_t | keys 0..t));
#                 x2 = LN2(x1 + CrossAttn(x1, g_t));  x3 = LN3(x2 + FF(x2));
#                 m_l,t = mean_{s<=t} x3_s;  p_l,t = W_p,l m_l,t + b;  g_t <- g_t + W_gu m_l,t + b
#   features_t = final_aggregation([p_0,t | ... | g_t]);  heads on [frac_grad(features_t) |
#   to_state_embed(s_t) (| latent)] — FractalWorldModelActorCritic.forward (:549-619) per timestep.
# Usable as OracleLearner's model (same forward contract as ref_port.OracleWMAC, a streaming cache).
# ----------------------------------------------------------------------------------------------

from torch import nn  # noqa: E402


class _OAttn(nn.Module):
    def __init__(self, d, inner):
        super().__init__()
        self.to_q, self.to_k = nn.Linear(d, inner, bias=False), nn.Linear(d, inner, bias=False)
        self.to_v, self.to_out = nn.Linear(d, inner, bias=False), nn.Linear(inner, d, bias=False)


class _OFF(nn.Module):
    def __init__(self, d, mult):
        super().__init__()
        self.ff = nn.Sequential(nn.Sequential(nn.Linear(d, d * mult), nn.GELU()), nn.Identity(),
                                nn.Linear(d * mult, d))


class _OBlock(nn.Module):
    def __init__(self, d, inner, mult):
        super().__init__()
        self.self_attn, self.global_attn, self.ff = _OAttn(d, inner), _OAttn(d, inner), _OFF(d, mult)
        self.norm1, self.norm2, self.norm3 = nn.LayerNorm(d), nn.LayerNorm(d), nn.LayerNorm(d)


class _OLevelEmb(nn.Module):
    def __init__(self, levels, d):
        super().__init__()
        self.level_embeds = nn.Parameter(torch.zeros(levels, d))
        pos = torch.arange(levels, dtype=torch.float32)[:, None]
        div = torch.exp(torch.arange(0, d, 2, dtype=torch.float32) * -(math.log(10000.0) / d))
        se = torch.zeros(levels, d)
        se[:, 0::2], se[:, 1::2] = torch.sin(pos * div), torch.cos(pos * div)
        self.register_buffer('scale_embeds', se)


class _OEncoder(nn.Module):
    def __init__(self, S, d, levels, inner, mult):
        super().__init__()
        self.input_embed = nn.Linear(S, d)
        self.level_embedding = _OLevelEmb(levels, d)
        self.global_state_init = nn.Parameter(torch.zeros(1, 1, d))
        self.global_state_update = nn.Linear(d, d)
        self.fractal_blocks = nn.ModuleList([_OBlock(d, inner, mult) for _ in range(levels)])
        self.upscale_layers = nn.ModuleList([nn.Linear(d, d) for _ in range(levels - 1)])
        self.downscale_layers = nn.ModuleList([nn.Linear(d, d) for _ in range(levels - 1)])
        self.level_projections = nn.ModuleList([nn.Linear(d, d) for _ in range(levels)])
        self.final_aggregation = nn.Sequential(nn.Linear(d * (levels + 1), 2 * d), nn.ReLU(), nn.Linear(2 * d, d))


class OracleFractalPolicy(nn.Module):
    """Causal fractal actor-critic on the reference's parameter names (fractal_rl.py:349-446 layout,
    separate blocks per level).  ``cfg``: oracle.ref_port.ModelConfig."""

    def __init__(self, cfg, levels, ff_mult=None):
        ff_mult = getattr(cfg, 'ff_mult', 4) if ff_mult is None else ff_mult
        super().__init__()
        from . import thirdparty as tp
        self.cfg, self.levels = cfg, levels
        d, S = cfg.dim, cfg.state_dim
        self.heads, self.dim_head = cfg.heads, cfg.dim_head
        self.fractal_encoder = _OEncoder(S, d, levels, cfg.heads * cfg.dim_head, ff_mult)
        self.reward_embed = nn.Parameter(torch.ones(d) * 1e-2)
        if cfg.continuous:
            self.action_embeds = nn.Linear(cfg.num_actions, d)
        else:
            self.action_embeds = nn.Module()
            self.action_embeds.embed = nn.Embedding(cfg.num_actions, d)
        self.to_state_embed = nn.Linear(S, d)
        self.to_pred_done = nn.Sequential(nn.Linear(2 * d, 1))
        self.to_pred = nn.Sequential(nn.Linear(2 * d, d), nn.SiLU(), nn.Linear(d, 2 * (S + 1)))
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
        from . import ref_port as R
        return R.safe_embed(self.action_embeds.embed.weight, actions)

    def _step(self, s_t, cache, key_mask=None):
        """One position for every row: s_t [b, S]; cache holds per level the K / V rows so far
        [b, H, t, dh] and the running sums of the level outputs [b, d].  key_mask [b, t + 1]: the
        key-padding mask of a padded minibatch (the learn step's attention masks keys past each
        episode's length, as x-transformers' mask does for the decoder)."""
        enc = self.fractal_encoder
        b = s_t.shape[0]
        H, dh = self.heads, self.dim_head
        t = cache['t']
        x = enc.input_embed(s_t)
        g = enc.global_state_init.reshape(1, -1).expand(b, -1)
        projs = []
        for li, blk in enumerate(enc.fractal_blocks):
            le = enc.level_embedding
            x = x + le.level_embeds[li] + le.scale_embeds[li]
            sa = blk.self_attn
            q, k, v = (m(x).view(b, H, 1, dh) for m in (sa.to_q, sa.to_k, sa.to_v))
            K = k if t == 0 else torch.cat((cache['k'][li], k), dim=2)
            V = v if t == 0 else torch.cat((cache['v'][li], v), dim=2)
            cache['k'][li], cache['v'][li] = K, V
            sim = (q @ K.transpose(-1, -2)) / math.sqrt(dh)
            if key_mask is not None:
                sim = sim.masked_fill(~key_mask[:, None, None, :], -torch.finfo(sim.dtype).max)
            a = sim.softmax(dim=-1) @ V
            x1 = blk.norm1(x + sa.to_out(a.reshape(b, H * dh)))
            ga = blk.global_attn    # attention of the row over the one global-state token
            gq, gk, gv = ga.to_q(x1).view(b, H, 1, dh), ga.to_k(g).view(b, H, 1, dh), ga.to_v(g).view(b, H, 1, dh)
            ca = ((gq @ gk.transpose(-1, -2)) / math.sqrt(dh)).softmax(dim=-1) @ gv
            x2 = blk.norm2(x1 + ga.to_out(ca.reshape(b, H * dh)))
            ff = blk.ff.ff
            x3 = blk.norm3(x2 + ff[2](F.gelu(ff[0][0](x2))))
            cache['sums'][li] = x3 if t == 0 else cache['sums'][li] + x3
            mean = cache['sums'][li] / (t + 1)
            projs.append(enc.level_projections[li](mean))
            g = g + enc.global_state_update(mean)
            x = x3
        cache['t'] = t + 1
        return enc.final_aggregation(torch.cat(projs + [g], dim=-1))

    def forward(self, state, actions=None, rewards=None, next_actions=None, latent_gene=None, mask=None, cache=None,
                reward_keep=True):
        """ref_port.OracleWMAC's contract.  The encoder reads the states only (as the reference's
        FractalWorldModelActorCritic.forward); ``cache`` continues a stream position by position."""
        from . import ref_port as R
        b, n, _ = state.shape
        if cache is None:
            cache = dict(t=0, k=[None] * self.levels, v=[None] * self.levels, sums=[None] * self.levels)
        t0 = cache['t']
        if mask is not None:
            assert t0 == 0, 'a key-padding mask applies to a whole sequence'
        feats = torch.stack([self._step(state[:, i], cache, None if mask is None else mask[:, :i + 1])
                             for i in range(n)], dim=1)
        state_pred = dones = None
        if next_actions is not None:
            ewa = torch.cat((feats, self.embed_actions(next_actions)), dim=-1)
            mean, var = R.continuous_params(self.to_pred(ewa))
            state_pred = torch.stack((mean, var))
            dones = self.to_pred_done(ewa)[..., 0].sigmoid()
        feats = R.frac_gradient(feats, self.cfg.frac_head_grad)
        ac_in = torch.cat((feats, self.to_state_embed(state)), dim=-1)
        if self.cfg.evolutionary:
            lat = self.latent_to_embed(latent_gene)
            if lat.ndim == 2:
                lat = lat[:, None, :].expand(-1, n, -1)
            ac_in = torch.cat((ac_in, lat), dim=-1)
        return self.action_head(ac_in), self.critic_head(ac_in), state_pred, dones, cache
