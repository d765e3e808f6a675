"""Restatements of the third-party libraries the reference hot path calls — TEST INFRASTRUCTURE.

None of these packages is present in this container, so their arithmetic is
restated from their published behaviour and is PARITY UNPINNED.  Every choice that cannot be
checked here is a named switch (defaults = best knowledge, recorded in DESIGN.md "decision log").

  x-transformers >=2.3.12      ContinuousTransformerWrapper + Decoder (pre-norm, rotary on dh//2
                               interleaved dims, gated values, learned value-residual mix, GELU FF)
                               reference call sites: x_transformers_rl.py:721-734 (build),
                               x_transformers_rl.py:505-512 (call; learn with mask, rollout with cache)
  hl-gauss-pytorch (unpinned)  HLGaussLoss  — x_transformers_rl.py:356-361, 427, 454-462, 843
  assoc-scan (unpinned)        AssocScan    — x_transformers_rl.py:634-636
  ema-pytorch (unpinned)       EMA          — x_transformers_rl.py:747, 753, 1194, 1269
  adam-atan2-pytorch           AdoptAtan2   — x_transformers_rl.py:749
  einx >=0.3.0                 multiply / less / where, only the patterns the reference uses

The module classes keep upstream parameter names so a state_dict made here has the reference's
key layout (the committed fractal checkpoints confirm to_q/to_k/to_v/to_out bias-free and
ff.ff.0.0 / ff.ff.2 with bias).

These classes double as ``sys.modules`` stand-ins when tests/golden/make_golden.py runs the
reference's own code to produce golden vectors.
"""
from __future__ import annotations

import math
from copy import deepcopy
from dataclasses import dataclass

import torch
import torch.nn.functional as F
from torch import nn

# --------------------------------------------------------------------------------------------
# switches for the unpinned x-transformers semantics
# --------------------------------------------------------------------------------------------


@dataclass
class XTConfig:
    # 'zero': rollout feeds one token per call, so upstream computes rotary positions as
    #         arange(x.shape[1]) = [0] -> rotary is the identity during cached decode (best
    #         knowledge).  'absolute': position = cache length (self-consistent
    #         with the full-sequence forward).
    rollout_rotary: str = 'zero'
    # direction of the value-residual lerp: 'toward_first' = v.lerp(v_first, mix)
    value_residual_lerp: str = 'toward_first'
    project_in_bias: bool = False


XT = XTConfig()


# --------------------------------------------------------------------------------------------
# einx subset (only the exact patterns x_transformers_rl.py uses)
# --------------------------------------------------------------------------------------------


class _EinxStub:
    """einx.multiply / less / where restricted to the patterns used at
    x_transformers_rl.py:194, 437-438, 499, 909 and distributed.py:93."""

    @staticmethod
    def multiply(pattern, a, b):
        p = pattern.replace(' ', '')
        if p == '...,d->...d':              # rewards (...) x reward_embed (d)
            return a[..., None] * b
        if p == 'bn...,bn->bn...':          # ratios (b n ...) x advantages (b n)
            extra = a.ndim - b.ndim
            return a * b.reshape(*b.shape, *((1,) * extra))
        raise NotImplementedError(pattern)

    @staticmethod
    def less(pattern, a, b):
        p = pattern.replace(' ', '')
        if p == 'n,b->bn':
            return a[None, :] < b[:, None]
        if p == 'ji->(ij)':
            return (a[None, :] < b[:, None]).reshape(-1)
        raise NotImplementedError(pattern)

    @staticmethod
    def where(pattern, cond, a, b):
        p = pattern.replace(' ', '')
        if p in ('bn,bnd,->bnd', 'bn,bnd,'):
            return torch.where(cond[..., None], a, torch.as_tensor(b, dtype=a.dtype))
        raise NotImplementedError(pattern)


einx = _EinxStub()


# --------------------------------------------------------------------------------------------
# assoc-scan: h_t = g_t * h_{t+1} + x_t (reverse), h_n = 0, along dim 1 — sequential order
# --------------------------------------------------------------------------------------------


class AssocScan(nn.Module):
    def __init__(self, reverse=False, use_accelerated=False, **kwargs):
        super().__init__()
        self.reverse = reverse

    def forward(self, gates, inputs):
        n = inputs.shape[1]
        out = torch.empty_like(inputs)
        h = torch.zeros_like(inputs[:, 0])
        order = range(n - 1, -1, -1) if self.reverse else range(n)
        for t in order:
            h = gates[:, t] * h + inputs[:, t]
            out[:, t] = h
        return out


# --------------------------------------------------------------------------------------------
# hl-gauss-pytorch
# --------------------------------------------------------------------------------------------


class HLGaussLoss(nn.Module):
    """Histogram loss with a Gaussian target (Farebrother et al. 2024).

    value(logits)          = sum(softmax(logits) * centres)
    loss(logits, target)   = cross_entropy(logits, normalised erf-histogram of N(target, sigma))
    Unpinned: ``reduction`` default ('mean' per upstream README usage ``loss.backward()``) and
    ``sigma`` default (sigma_to_bin_ratio * bin_width, ratio 2.0)."""

    default_reduction = 'mean'
    default_sigma_ratio = 2.0

    def __init__(self, min_value, max_value, num_bins, sigma=None, sigma_to_bin_ratio=None,
                 clamp_to_range=False):
        super().__init__()
        self.min_value, self.max_value, self.num_bins = float(min_value), float(max_value), num_bins
        support = torch.linspace(min_value, max_value, num_bins + 1, dtype=torch.float32)
        bin_size = (self.max_value - self.min_value) / num_bins
        ratio = self.default_sigma_ratio if sigma_to_bin_ratio is None else sigma_to_bin_ratio
        self.sigma = sigma if sigma is not None else ratio * bin_size
        self.clamp_to_range = clamp_to_range
        self.register_buffer('support', support, persistent=False)
        self.register_buffer('centers', (support[:-1] + support[1:]) / 2, persistent=False)

    def target_probs(self, target):
        if self.clamp_to_range:
            target = target.clamp(self.min_value, self.max_value)
        cdf = torch.special.erf((self.support - target[..., None]) / (math.sqrt(2.0) * self.sigma))
        z = cdf[..., -1] - cdf[..., 0]
        return (cdf[..., 1:] - cdf[..., :-1]) / z[..., None]

    def forward(self, logits, target=None, reduction=None):
        if target is None:
            return (logits.softmax(dim=-1) * self.centers).sum(dim=-1)
        reduction = self.default_reduction if reduction is None else reduction
        tp = self.target_probs(target)
        per = -(tp * logits.log_softmax(dim=-1)).sum(dim=-1)
        if reduction == 'none':
            return per
        if reduction == 'mean':
            return per.mean()
        return per.sum()


# --------------------------------------------------------------------------------------------
# x-transformers: ContinuousTransformerWrapper + Decoder (module classes with upstream names)
# --------------------------------------------------------------------------------------------


class LayerNorm(nn.Module):
    """x-transformers LayerNorm: F.layer_norm without affine, times a learned gamma (no beta)."""

    def __init__(self, dim):
        super().__init__()
        self.dim = dim
        self.gamma = nn.Parameter(torch.ones(dim))

    def forward(self, x):
        return F.layer_norm(x, (self.dim,), eps=1e-5) * self.gamma


class RMSNorm(nn.Module):
    """x-transformers RMSNorm (Decoder use_rmsnorm): F.normalize(x, dim=-1) * dim ** 0.5 * g (no
    unit offset); parameter ``g``."""

    def __init__(self, dim):
        super().__init__()
        self.scale = dim ** 0.5
        self.g = nn.Parameter(torch.ones(dim))

    def forward(self, x):
        return F.normalize(x, dim=-1) * self.scale * self.g


class RotaryEmbedding(nn.Module):
    """x-transformers RotaryEmbedding; ``use_xpos`` (Decoder rotary_xpos): the xPos scale
    ((arange(0, dim, 2) + 0.4 dim) / (1.4 dim)) ** ((pos - max_pos // 2) / scale_base), max_pos =
    pos.max() + 1, interleaved like the frequencies (q times it, k divided by it; x-transformers
    apply_rotary_pos_emb).  The scale table is a non-persistent buffer here (parity unpinned)."""

    def __init__(self, dim, base=10000., use_xpos=False, scale_base=512.):
        super().__init__()
        inv_freq = 1. / (base ** (torch.arange(0, dim, 2).float() / dim))
        self.register_buffer('inv_freq', inv_freq)
        self.use_xpos, self.scale_base = use_xpos, scale_base
        self.register_buffer('xpos_scale', (torch.arange(0, dim, 2).float() + 0.4 * dim) / (1.4 * dim),
                             persistent=False)

    def forward(self, pos):
        freqs = pos.float()[:, None] * self.inv_freq[None, :]
        return torch.stack((freqs, freqs), dim=-1).reshape(pos.shape[0], -1)   # interleaved

    def xpos(self, pos):
        """The per-(position, channel) xPos factor for q (k takes its inverse), or None."""
        if not self.use_xpos:
            return None
        power = (pos.float() - (int(pos.max()) + 1) // 2) / self.scale_base
        sc = self.xpos_scale[None, :] ** power[:, None]
        return torch.stack((sc, sc), dim=-1).reshape(pos.shape[0], -1)


def rotate_half(x):
    x = x.reshape(*x.shape[:-1], -1, 2)
    x1, x2 = x.unbind(-1)
    return torch.stack((-x2, x1), dim=-1).reshape(*x.shape[:-2], -1)


def apply_rotary(t, freqs, scale=1.):
    rot = freqs.shape[-1]
    tr, tu = t[..., :rot], t[..., rot:]
    tr = tr * freqs.cos() * scale + rotate_half(tr) * freqs.sin() * scale
    return torch.cat((tr, tu), dim=-1)


class _Rearrange(nn.Module):
    def forward(self, x):           # 'b n h -> b h n 1'
        return x.permute(0, 2, 1).unsqueeze(-1)


class Attention(nn.Module):
    """``qk_norm`` (Decoder attn_qk_norm): q and k l2-normalised per head (F.normalize) after the
    projections and before the rotary, the scores scaled by ``qk_norm_scale`` instead of dh ** -0.5
    (x-transformers Attention qk_norm, qk_norm_groups = 1, no dim scale)."""

    def __init__(self, dim, heads, dim_head, dropout=0., gate_values=True, learned_value_residual_mix=False,
                 qk_norm=False, qk_norm_scale=10.):
        super().__init__()
        inner = heads * dim_head
        self.heads, self.dim_head = heads, dim_head
        self.qk_norm, self.qk_norm_scale = qk_norm, qk_norm_scale
        self.to_q = nn.Linear(dim, inner, bias=False)
        self.to_k = nn.Linear(dim, inner, bias=False)
        self.to_v = nn.Linear(dim, inner, bias=False)
        self.to_out = nn.Linear(inner, dim, bias=False)
        self.attn_dropout = nn.Dropout(dropout)
        self.to_v_gate = None
        if gate_values:
            self.to_v_gate = nn.Linear(dim, inner)
            nn.init.constant_(self.to_v_gate.weight, 0.)
            nn.init.constant_(self.to_v_gate.bias, 10.)
        self.to_value_residual_mix = None
        if learned_value_residual_mix:
            self.to_value_residual_mix = nn.Sequential(nn.Linear(dim, heads), nn.Sigmoid(), _Rearrange())
            nn.init.zeros_(self.to_value_residual_mix[0].weight)
            nn.init.zeros_(self.to_value_residual_mix[0].bias)

    def forward(self, x, freqs, key_mask=None, cache_kv=None, value_residual=None, xpos=None):
        b, n, _ = x.shape
        h, dh = self.heads, self.dim_head
        split = lambda t: t.reshape(b, n, h, dh).permute(0, 2, 1, 3)
        q, k, v = split(self.to_q(x)), split(self.to_k(x)), split(self.to_v(x))
        orig_v = v
        if value_residual is not None and self.to_value_residual_mix is not None:
            mix = self.to_value_residual_mix(x)
            if XT.value_residual_lerp == 'toward_first':
                v = v.lerp(value_residual, mix)
            else:
                v = value_residual.lerp(v, mix)
        scale = dh ** -0.5
        if self.qk_norm:
            q, k = F.normalize(q, dim=-1), F.normalize(k, dim=-1)
            scale = self.qk_norm_scale
        if freqs is not None:
            xq, xk = (1., 1.) if xpos is None else (xpos, xpos ** -1.)
            q, k = apply_rotary(q, freqs, xq), apply_rotary(k, freqs, xk)
        if cache_kv is not None:
            k = torch.cat((cache_kv[0], k), dim=-2)
            v = torch.cat((cache_kv[1], v), dim=-2)
        i, j = q.shape[-2], k.shape[-2]
        sim = torch.einsum('bhid,bhjd->bhij', q, k) * scale
        neg = -torch.finfo(sim.dtype).max
        causal = torch.ones((i, j), dtype=torch.bool, device=x.device).triu(j - i + 1)
        sim = sim.masked_fill(causal, neg)
        if key_mask is not None:
            sim = sim.masked_fill(~key_mask[:, None, None, :], neg)
        attn = self.attn_dropout(sim.softmax(dim=-1, dtype=torch.float32))
        out = torch.einsum('bhij,bhjd->bhid', attn, v)
        out = out.permute(0, 2, 1, 3).reshape(b, n, h * dh)
        if self.to_v_gate is not None:
            out = out * self.to_v_gate(x).sigmoid()
        return self.to_out(out), (k, v), orig_v


class GLU(nn.Module):
    """x-transformers GLU (the ``ff_glu`` project-in): ``proj`` = Linear(dim, 2 inner) (always with a
    bias), ``x, gate = proj(x).chunk(2, -1)``, out = x * act(gate) (no mult_bias)."""

    def __init__(self, dim_in, dim_out, activation):
        super().__init__()
        self.act = activation
        self.proj = nn.Linear(dim_in, dim_out * 2)

    def forward(self, x):
        x, gate = self.proj(x).chunk(2, dim=-1)
        return x * self.act(gate)


class FeedForward(nn.Module):
    """x-transformers FeedForward (GELU); ``no_bias``: the Linears without bias (ff_no_bias; the GLU
    projection keeps its bias); ``glu``: the GLU project-in (ff_glu)."""

    def __init__(self, dim, mult=4, dropout=0., no_bias=False, glu=False):
        super().__init__()
        inner = dim * mult
        project_in = (GLU(dim, inner, nn.GELU()) if glu else
                      nn.Sequential(nn.Linear(dim, inner, bias=not no_bias), nn.GELU()))
        self.ff = nn.Sequential(project_in, nn.Dropout(dropout), nn.Linear(inner, dim, bias=not no_bias))

    def forward(self, x):
        return self.ff(x)


class XAttention(nn.Module):
    """x-transformers ``Attention`` as fractal_rl.py builds and calls it (:87-102, :123, :127):
    ``Attention(dim, heads, dim_head, dropout, dim_context=None)``, ``forward(x, context=None,
    mask=None)``; not causal, no rotary, no gates.  q from x, k / v from ``context`` (default x);
    ``mask`` masks keys only when there is no context (upstream: ``input_mask = context_mask``, else
    ``mask`` for self-attention), by -finfo.max; post-softmax dropout; heads merged, ``to_out``."""

    def __init__(self, dim, heads=8, dim_head=64, dropout=0., dim_context=None, **unsupported):
        super().__init__()
        if unsupported:
            raise NotImplementedError(f'restated Attention does not model {sorted(unsupported)}')
        inner, ctx = heads * dim_head, dim_context or dim
        self.heads, self.dim_head = heads, dim_head
        self.to_q = nn.Linear(dim, inner, bias=False)
        self.to_k = nn.Linear(ctx, inner, bias=False)
        self.to_v = nn.Linear(ctx, inner, bias=False)
        self.to_out = nn.Linear(inner, dim, bias=False)
        self.attn_dropout = nn.Dropout(dropout)

    def forward(self, x, context=None, mask=None, context_mask=None):
        b, i, _ = x.shape
        kv = x if context is None else context
        j = kv.shape[1]
        h, dh = self.heads, self.dim_head
        q = self.to_q(x).reshape(b, i, h, dh).transpose(1, 2)
        k = self.to_k(kv).reshape(b, j, h, dh).transpose(1, 2)
        v = self.to_v(kv).reshape(b, j, h, dh).transpose(1, 2)
        sim = q @ k.transpose(-1, -2) * dh ** -0.5
        key_mask = context_mask if context is not None else mask
        if key_mask is not None:
            sim = sim.masked_fill(~key_mask[:, None, None, :], -torch.finfo(sim.dtype).max)
        out = self.attn_dropout(sim.softmax(dim=-1)) @ v
        return self.to_out(out.transpose(1, 2).reshape(b, i, h * dh))


class _Residual(nn.Module):
    def forward(self, out, residual):
        return out + residual


class _AttnCache:
    def __init__(self, cached_kv):
        self.cached_kv = cached_kv


class LayerIntermediates:
    """What x-transformers returns as ``intermediates`` and accepts back as ``cache``."""

    def __init__(self, attn_intermediates, cache_length):
        self.attn_intermediates = attn_intermediates
        self.cache_length = cache_length


class Decoder(nn.Module):
    def __init__(self, dim, depth, heads=8, attn_dim_head=64, rotary_pos_emb=False, attn_dropout=0.,
                 ff_dropout=0., verbose=True, attn_gate_values=False, add_value_residual=False,
                 learned_value_residual_mix=False, ff_mult=4, ff_no_bias=False, ff_glu=False, attn_qk_norm=False,
                 attn_qk_norm_scale=10., rotary_xpos=False, rotary_xpos_scale_base=512., use_rmsnorm=False,
                 **unsupported):
        super().__init__()
        if unsupported:
            raise NotImplementedError(f'restated Decoder does not model {sorted(unsupported)}')
        self.dim, self.depth, self.causal = dim, depth, True
        self.add_value_residual = add_value_residual
        self.layers = nn.ModuleList()
        Norm = RMSNorm if use_rmsnorm else LayerNorm
        for ind in range(depth):
            attn = Attention(dim, heads, attn_dim_head, attn_dropout, attn_gate_values,
                             learned_value_residual_mix=learned_value_residual_mix and add_value_residual and ind > 0,
                             qk_norm=attn_qk_norm, qk_norm_scale=attn_qk_norm_scale)
            self.layers.append(nn.ModuleList([nn.ModuleList([Norm(dim), None, None]), attn, _Residual()]))
            self.layers.append(nn.ModuleList([nn.ModuleList([Norm(dim), None, None]),
                                              FeedForward(dim, ff_mult, ff_dropout, ff_no_bias, ff_glu), _Residual()]))
        self.rotary_pos_emb = RotaryEmbedding(attn_dim_head // 2, use_xpos=rotary_xpos,
                                              scale_base=rotary_xpos_scale_base) if rotary_pos_emb else None
        self.final_norm = Norm(dim)

    def forward(self, x, mask=None, cache: LayerIntermediates | None = None):
        n = x.shape[1]
        prev = 0 if cache is None else cache.cache_length
        freqs = xpos = None
        if self.rotary_pos_emb is not None:
            if cache is not None and XT.rollout_rotary == 'absolute':
                pos = torch.arange(prev, prev + n, device=x.device)
            else:
                pos = torch.arange(n, device=x.device)
            freqs = self.rotary_pos_emb(pos)
            xpos = self.rotary_pos_emb.xpos(pos)
        caches = iter(cache.attn_intermediates) if cache is not None else None
        new_caches = []
        first_values = None
        for norms, block, residual in self.layers:
            res = x
            xn = norms[0](x)
            if isinstance(block, Attention):
                ckv = next(caches).cached_kv if caches is not None else None
                out, kv, orig_v = block(xn, freqs, key_mask=mask, cache_kv=ckv,
                                        value_residual=first_values if self.add_value_residual else None, xpos=xpos)
                if first_values is None:
                    first_values = orig_v
                new_caches.append(_AttnCache(kv))
            else:
                out = block(xn)
            x = residual(out, res)
        return self.final_norm(x), LayerIntermediates(new_caches, prev + n)


class ContinuousTransformerWrapper(nn.Module):
    def __init__(self, *, dim_in, dim_out, max_seq_len, attn_layers, probabilistic=False, **unsupported):
        super().__init__()
        if unsupported:
            raise NotImplementedError(f'restated wrapper does not model {sorted(unsupported)}')
        self.attn_layers = attn_layers
        self.max_seq_len = max_seq_len
        self.project_in = nn.Linear(dim_in, attn_layers.dim, bias=XT.project_in_bias)

    def forward(self, x, mask=None, cache=None, sum_embeds=None, return_embeddings=False,
                return_intermediates=False, **unused):
        assert return_embeddings, 'the reference only uses return_embeddings=True'
        x = self.project_in(x)
        if sum_embeds is not None:
            x = x + sum_embeds
        x, inter = self.attn_layers(x, mask=mask, cache=cache)
        return (x, inter) if return_intermediates else x


# --------------------------------------------------------------------------------------------
# ema-pytorch
# --------------------------------------------------------------------------------------------


class EMA(nn.Module):
    """Restated subset of ema-pytorch's EMA (update_after_step=100, update_every=10,
    inv_gamma=1, power=2/3, min_value=0 defaults)."""

    def __init__(self, model, beta=0.9999, update_after_step=100, update_every=10, inv_gamma=1.,
                 power=2 / 3, min_value=0., include_online_model=True, forward_method_names=(),
                 update_model_with_ema_every=None, update_model_with_ema_beta=0.):
        super().__init__()
        self.beta = beta
        self.online = [model] if not include_online_model else None
        if include_online_model:
            self.online_model = model
        self.ema_model = deepcopy(model)
        self.ema_model.requires_grad_(False)
        self.update_after_step, self.update_every = update_after_step, update_every
        self.inv_gamma, self.power, self.min_value = inv_gamma, power, min_value
        self.update_model_with_ema_every = update_model_with_ema_every
        self.update_model_with_ema_beta = update_model_with_ema_beta
        for name in forward_method_names:
            setattr(self, name, getattr(self.ema_model, name))
        self.register_buffer('step', torch.tensor(0))
        self.register_buffer('initted', torch.tensor(False))

    @property
    def model(self):
        return self.online[0] if self.online is not None else self.online_model

    def current_decay(self):
        epoch = max(self.step.item() - self.update_after_step - 1, 0)
        if epoch <= 0:
            return 0.
        value = 1 - (1 + epoch / self.inv_gamma) ** -self.power
        return min(max(value, self.min_value), self.beta)

    @torch.no_grad()
    def copy_params_from_model_to_ema(self):
        for pe, pm in zip(self.ema_model.parameters(), self.model.parameters()):
            pe.copy_(pm)
        for be, bm in zip(self.ema_model.buffers(), self.model.buffers()):
            be.copy_(bm)

    @torch.no_grad()
    def update(self):
        step = self.step.item()
        self.step += 1
        should_update = step % self.update_every == 0
        if should_update and step <= self.update_after_step:
            self.copy_params_from_model_to_ema()
            return
        if should_update:
            if not self.initted.item():
                self.copy_params_from_model_to_ema()
                self.initted.fill_(True)
            decay = self.current_decay()
            for pe, pm in zip(self.ema_model.parameters(), self.model.parameters()):
                pe.lerp_(pm, 1. - decay)
        # the online-model copy-back is checked on every step, outside should_update (ema-pytorch)
        if self.update_model_with_ema_every is not None and step % self.update_model_with_ema_every == 0:
            for pe, pm in zip(self.ema_model.parameters(), self.model.parameters()):
                pm.lerp_(pe, 1. - self.update_model_with_ema_beta)

    def add_to_optimizer_post_step_hook(self, optimizer):
        return optimizer.register_step_post_hook(lambda *_: self.update())

    @torch.no_grad()
    def forward_eval(self, *args, **kwargs):
        training = self.ema_model.training
        self.ema_model.eval()
        out = self.ema_model(*args, **kwargs)
        self.ema_model.train(training)
        return out

    def forward(self, *args, **kwargs):
        return self.ema_model(*args, **kwargs)


# --------------------------------------------------------------------------------------------
# adam-atan2-pytorch: AdoptAtan2
# --------------------------------------------------------------------------------------------


class AdoptAtan2(torch.optim.Optimizer):
    """ADOPT (Taniguchi et al. 2024) with the atan2 update of Everett et al. 2024, decoupled weight
    decay, regenerative regularisation (Kumar et al. 2023) and the cautious mask (Liang et al. 2024).

    step (per tensor p, grad g):
      first step : v = g^2, m = 0 (no parameter update)
      later      : u = atan2(g, b*sqrt(v)); m = lerp(m, u, 1-beta1)
                   cautious: scale = where(u*g > 0, 1, c) / mean(...) ; p -= lr * a * m * scale
                   v = lerp(v, g^2, 1-beta2)
    regen: p = lerp(p, p_init, lr/init_lr * regen_rate) before the update."""

    def __init__(self, params, lr=1e-4, betas=(0.9, 0.99), weight_decay=0., regen_reg_rate=0.,
                 decoupled_wd=True, cautious_factor=1., a=1.27, b=1.):
        defaults = dict(lr=lr, betas=betas, a=a, b=b, weight_decay=weight_decay,
                        regen_reg_rate=regen_reg_rate, cautious_factor=cautious_factor)
        super().__init__(params, defaults)
        self._init_lr = lr
        self.decoupled_wd = decoupled_wd

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            lr, wd, regen, cf = group['lr'], group['weight_decay'], group['regen_reg_rate'], group['cautious_factor']
            beta1, beta2 = group['betas']
            a, b = group['a'], group['b']
            if self.decoupled_wd:
                wd = wd / self._init_lr
            for p in group['params']:
                if p.grad is None:
                    continue
                g = p.grad
                state = self.state[p]
                if regen > 0. and 'param_init' in state:
                    p.lerp_(state['param_init'], lr / self._init_lr * regen)
                if wd > 0.:
                    p.mul_(1. - lr * wd)
                if len(state) == 0:
                    state['steps'] = 0
                    state['m'] = torch.zeros_like(g)
                    state['v'] = g * g
                    if regen > 0.:
                        state['param_init'] = p.clone()
                    continue
                m, v = state['m'], state['v']
                update = g.atan2(b * v.sqrt())
                m.lerp_(update, 1. - beta1)
                upd = m
                if cf < 1.:
                    align = (m * g) > 0
                    scale = torch.where(align, torch.ones_like(g), torch.full_like(g, cf))
                    scale = scale / scale.mean().clamp(min=1e-5)
                    upd = m * scale
                p.add_(upd * a, alpha=-lr)
                v.lerp_(g * g, 1. - beta2)
                state['steps'] += 1
        return loss
