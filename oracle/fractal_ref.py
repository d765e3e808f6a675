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
    """FractalProcessingBlock.forward (fractal_rl.py:120-136), use_global_attention=True."""
    x = _layernorm(x + _attention(x, x, sd, pre + '.self_attn', heads, dim_head, key_mask), sd, pre + '.norm1')
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
