"""WorldModelActorCritic for the MI355X learner.

Parameter names and shapes follow the reference state_dict (x_transformers_rl.py:281-392 with the
x-transformers ContinuousTransformerWrapper/Decoder inside), so checkpoints interchange with
``Agent.save`` / ``Agent.load`` of the reference (xtrl.py:792-806).

Compute: the rollout never calls this module — it runs the packed weights through
libxtrl_hip's decode step (rollout.py).  The learn step (``forward_train``) keeps PyTorch autograd
for the dense layers and routes the attention core through the HIP flash kernel (ops.attention)
and the losses through the fused HIP loss (ops.fused_loss).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn.functional as F
from torch import nn

from . import ops


@dataclass
class ModelConfig:
    state_dim: int
    num_actions: int
    dim: int = 48
    depth: int = 1
    heads: int = 4
    dim_head: int = 16
    num_bins: int = 100
    reward_range: tuple = (-1., 1.)
    continuous: bool = False
    squash: bool = True
    evolutionary: bool = False
    dim_gene: int = 0
    frac_head_grad: float = 0.5
    entropy_weight: float = 0.01
    eps_clip: float = 0.2
    value_clip: float = 0.4
    dropout: float = 0.25
    reward_dropout: float = 0.5
    gate_values: bool = False
    value_residual: bool = False
    learned_mix: bool = False
    ff_mult: int = 4
    ff_no_bias: bool = False             # x-transformers FeedForward no_bias (world_model['ff_no_bias'])
    ff_glu: bool = False                 # x-transformers FeedForward glu (world_model['ff_glu']): GELU-gated project-in
    rms_norm: bool = False               # x-transformers use_rmsnorm: RMSNorm pre-norms / final norm (param .g)
    qk_norm: bool = False                # x-transformers attn_qk_norm: q, k l2-normalised per head, scores x qk_norm_scale
    qk_norm_scale: float = 10.           # x-transformers attn_qk_norm_scale
    rotary_xpos: bool = False            # x-transformers rotary_xpos: xPos-scaled rotary (q x s^p, k / s^p)
    xpos_scale_base: float = 512.        # x-transformers rotary_xpos_scale_base
    rotary_abs_rollout: bool = False     # decision log: reference semantics = rotary position 0 in rollout
    hl_reduction_mean: bool = True       # decision log: hl-gauss-pytorch default reduction
    hl_sigma_ratio: float = 2.0

    @property
    def inner(self):
        return self.heads * self.dim_head

    @property
    def in_dim(self):
        return self.dim * (3 if self.evolutionary else 2)


class XLayerNorm(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.dim = dim
        self.gamma = nn.Parameter(torch.ones(dim))

    def forward(self, x):
        return F.layer_norm(x, (self.dim,), eps=1e-5) * self.gamma


class XRMSNorm(nn.Module):
    """x-transformers RMSNorm (Decoder use_rmsnorm): F.normalize(x, dim=-1) * sqrt(dim) * g."""

    def __init__(self, dim):
        super().__init__()
        self.dim = dim
        self.g = nn.Parameter(torch.ones(dim))

    def forward(self, x):
        return F.normalize(x, dim=-1) * self.dim ** 0.5 * self.g


def norm_gain(mod):
    """The gain of a decoder norm: LayerNorm.gamma or RMSNorm.g."""
    return mod.g if isinstance(mod, XRMSNorm) else mod.gamma


class XAttention(nn.Module):
    def __init__(self, c: ModelConfig, mix: bool):
        super().__init__()
        d, inner = c.dim, c.inner
        self.to_q = nn.Linear(d, inner, bias=False)
        self.to_k = nn.Linear(d, inner, bias=False)
        self.to_v = nn.Linear(d, inner, bias=False)
        self.to_out = nn.Linear(inner, d, bias=False)
        self.to_v_gate = None
        if c.gate_values:
            self.to_v_gate = nn.Linear(d, inner)
            nn.init.constant_(self.to_v_gate.weight, 0.)
            nn.init.constant_(self.to_v_gate.bias, 10.)
        self.to_value_residual_mix = None
        if mix:
            self.to_value_residual_mix = nn.Sequential(nn.Linear(d, c.heads))
            nn.init.zeros_(self.to_value_residual_mix[0].weight)
            nn.init.zeros_(self.to_value_residual_mix[0].bias)


class XGLU(nn.Module):
    """x-transformers GLU (FeedForward glu = True): proj = Linear(dim, 2 inner) with a bias (value
    rows, then gate rows), out = value * gelu(gate) — state_dict names ff.0.proj.*"""

    def __init__(self, dim, inner):
        super().__init__()
        self.proj = nn.Linear(dim, 2 * inner)


class XFeedForward(nn.Module):
    def __init__(self, c: ModelConfig):
        super().__init__()
        inner, bias = c.dim * c.ff_mult, not c.ff_no_bias
        project_in = XGLU(c.dim, inner) if c.ff_glu else nn.Sequential(nn.Linear(c.dim, inner, bias=bias), nn.GELU())
        self.ff = nn.Sequential(project_in, nn.Dropout(c.dropout), nn.Linear(inner, c.dim, bias=bias))


class _Residual(nn.Module):
    pass


class XDecoder(nn.Module):
    def __init__(self, c: ModelConfig):
        super().__init__()
        self.dim = c.dim
        self.layers = nn.ModuleList()
        Norm = XRMSNorm if c.rms_norm else XLayerNorm
        for ind in range(c.depth):
            mix = c.value_residual and c.learned_mix and ind > 0
            self.layers.append(nn.ModuleList([nn.ModuleList([Norm(c.dim), None, None]), XAttention(c, mix),
                                              _Residual()]))
            self.layers.append(nn.ModuleList([nn.ModuleList([Norm(c.dim), None, None]), XFeedForward(c),
                                              _Residual()]))
        self.rotary_pos_emb = nn.Module()
        rot = c.dim_head // 2
        self.rotary_pos_emb.register_buffer('inv_freq', 1. / (10000 ** (torch.arange(0, rot, 2).float() / rot)))
        self.final_norm = Norm(c.dim)


class XTransformer(nn.Module):
    def __init__(self, c: ModelConfig):
        super().__init__()
        self.attn_layers = XDecoder(c)
        self.project_in = nn.Linear(c.state_dim, c.dim, bias=False)


def _rotate_half(x):
    x = x.reshape(*x.shape[:-1], -1, 2)
    x1, x2 = x.unbind(-1)
    return torch.stack((-x2, x1), dim=-1).reshape(*x.shape[:-2], -1)


def bucket_ranges(buckets, flat):
    """[(start, end)] of each bucket (a list of name groups, in flat order) in ``flat.grad_ext``; the
    last one runs to its end: the RSNorm-mean tail rides with it."""
    out = []
    for b in buckets:
        names = [n for g in b for n in g]
        out.append([flat.index[names[0]][0], flat.index[names[-1]][1]] if names else None)
    for i in range(len(out)):
        if out[i] is None:
            out[i] = [out[i - 1][1], out[i - 1][1]] if i else [0, 0]
    for a, b in zip(out, out[1:]):
        assert a[1] == b[0], 'flat buckets are not contiguous'
    out[-1][1] = flat.grad_ext.numel()
    return [tuple(r) for r in out]


class WorldModelActorCritic(nn.Module):
    def __init__(self, c: ModelConfig):
        super().__init__()
        d = c.dim
        self.cfg = c
        self.transformer = XTransformer(c)
        self.reward_embed = nn.Parameter(torch.ones(d) * 1e-2)
        if c.continuous:
            self.action_embeds = nn.Linear(c.num_actions, d)
        else:
            self.action_embeds = nn.Module()
            self.action_embeds.embed = nn.Embedding(c.num_actions, d)
        self.to_state_embed = nn.Linear(c.state_dim, d)
        self.to_pred_done = nn.Sequential(nn.Linear(2 * d, 1))
        self.to_pred = nn.Sequential(nn.Linear(2 * d, d), nn.SiLU(), nn.Linear(d, 2 * (c.state_dim + 1)))
        if c.evolutionary:
            self.latent_to_embed = nn.Linear(c.dim_gene, d)
        n_out = c.num_actions * (2 if c.continuous else 1)
        self.critic_head = nn.Sequential(nn.Linear(c.in_dim, 2 * d), nn.SiLU(), nn.Linear(2 * d, c.num_bins))
        self.action_head = nn.Sequential(nn.Linear(c.in_dim, 2 * d), nn.SiLU(), nn.Linear(2 * d, n_out))
        lo, hi = c.reward_range
        support = torch.linspace(lo, hi, c.num_bins + 1, dtype=torch.float32)
        self.register_buffer('hl_support', support, persistent=False)
        self.register_buffer('hl_centers', (support[:-1] + support[1:]) / 2, persistent=False)
        self.hl_sigma = c.hl_sigma_ratio * (hi - lo) / c.num_bins

    # ---- pieces shared with the rollout weight packing -----------------------------------------
    def blocks(self):
        layers = self.transformer.attn_layers.layers
        return [(layers[2 * i], layers[2 * i + 1]) for i in range(len(layers) // 2)]

    def embed_actions(self, actions):
        if self.cfg.continuous:
            return self.action_embeds(actions)
        # SafeEmbedding (xtrl.py:181-195) as a one-hot product: its backward is a small GEMM
        # instead of a scatter-add of 16K rows into A rows
        onehot = F.one_hot(actions.clamp(min=0), self.cfg.num_actions).to(torch.float32)
        onehot = onehot * (actions >= 0)[..., None].to(torch.float32)
        return onehot @ self.action_embeds.embed.weight

    def _zero_bias(self, n, like):
        z = getattr(self, '_zb', None)
        if z is None or z.shape[0] < n or z.device != like.device:
            z = torch.zeros(max(n, 1024), device=like.device)
            self._zb = z
        return z[:n]

    def hl_value(self, logits):
        return (logits.softmax(dim=-1) * self.hl_centers).sum(-1)

    # ---- flat-buffer layout / binding ---------------------------------------------------------------
    def flat_buckets_names(self):
        """Parameter groups of the flat buffer, bucketed in the order the fused backward completes
        them (train.hip records an event per bucket, include/xtrl_hip.h grad_events): [heads + state /
        gene embeddings + final norm], [decoder block L-1], ..., [block 0], [input embeddings].  A
        group's names must be adjacent: the q|k|v|gate|mix weights of each attention block, the first
        actor / critic head layers and to_pred.0 | to_pred_done are one GEMM operand each (views).
        Groups whose size is not a multiple of 4 floats move to the last bucket, so every GEMM weight
        starts 16-byte aligned (float4 operand loads).  -> list of buckets, each a list of groups."""
        c = self.cfg
        params = dict(self.named_parameters())
        taken = set()

        def grp(names):
            taken.update(names)
            return list(names)

        heads = [grp(['action_head.0.weight', 'critic_head.0.weight']), grp(['action_head.0.bias', 'critic_head.0.bias']),
                 grp(['to_pred.0.weight', 'to_pred_done.0.weight']), grp(['to_pred.0.bias', 'to_pred_done.0.bias'])]
        head_pre = ('action_head.', 'critic_head.', 'to_pred.', 'to_pred_done.', 'to_state_embed.', 'latent_to_embed.',
                    'transformer.attn_layers.final_norm.')
        heads += [grp([n]) for n in params if n not in taken and n.startswith(head_pre)]
        blocks = []
        for li in reversed(range(len(self.blocks()))):
            pa, pf = f'transformer.attn_layers.layers.{2 * li}.', f'transformer.attn_layers.layers.{2 * li + 1}.'
            pre = pa + '1.'
            mix = c.value_residual and c.learned_mix and li > 0
            g = [grp([pre + 'to_q.weight', pre + 'to_k.weight', pre + 'to_v.weight']
                     + ([pre + 'to_v_gate.weight'] if c.gate_values else [])
                     + ([pre + 'to_value_residual_mix.0.weight'] if mix else []))]
            bias = ([pre + 'to_v_gate.bias'] if c.gate_values else []) + \
                   ([pre + 'to_value_residual_mix.0.bias'] if mix else [])
            if bias:
                g.append(grp(bias))
            g += [grp([n]) for n in params if n not in taken and (n.startswith(pa) or n.startswith(pf))]
            blocks.append(g)
        embeds = [grp([n]) for n in params if n not in taken]
        buckets = [heads] + blocks + [embeds]
        size = lambda g: sum(params[n].numel() for n in g)
        tail = [g for b in buckets for g in b if size(g) % 4]
        buckets = [[g for g in b if size(g) % 4 == 0] for b in buckets]
        buckets[-1] += tail
        return buckets

    def flat_order(self):
        return [n for b in self.flat_buckets_names() for g in b for n in g]

    def flat_bucket_ranges(self, flat):
        return bucket_ranges(self.flat_buckets_names(), flat)

    def bind_flat(self, flat, ws):
        """Record the concatenated weight / gradient views used by forward_train."""
        c = self.cfg
        d, I = c.dim, c.inner
        self._flat, self._ws = flat, ws
        self._proj = []
        for li, (_, _) in enumerate(self.blocks()):
            pre = f'transformer.attn_layers.layers.{2 * li}.1.'
            mix = c.value_residual and c.learned_mix and li > 0
            wn = [pre + 'to_q.weight', pre + 'to_k.weight', pre + 'to_v.weight']
            wn += [pre + 'to_v_gate.weight'] if c.gate_values else []
            wn += [pre + 'to_value_residual_mix.0.weight'] if mix else []
            bn = ([pre + 'to_v_gate.bias'] if c.gate_values else []) + ([pre + 'to_value_residual_mix.0.bias'] if mix else [])
            n_out = 3 * I + (I if c.gate_values else 0) + (c.heads if mix else 0)
            entry = dict(w=flat.span(wn).view(n_out, d), wg=flat.span(wn, flat.grad).view(n_out, d), mix=mix,
                         b=flat.span(bn) if bn else None, bg=flat.span(bn, flat.grad) if bn else None)
            self._proj.append(entry)
        hn = ['action_head.0.weight', 'critic_head.0.weight']
        bn = ['action_head.0.bias', 'critic_head.0.bias']
        self._head1 = dict(w=flat.span(hn).view(4 * d, c.in_dim), wg=flat.span(hn, flat.grad).view(4 * d, c.in_dim),
                           b=flat.span(bn), bg=flat.span(bn, flat.grad))

    def _lin(self, x, mod):
        b = mod.bias
        return ops.xlinear(x, mod.weight, b, mod.weight.grad, b.grad if b is not None else None, self._ws)

    # ---- learn-step forward (xtrl.py:479-559 with the mask path of x-transformers) --------------
    def forward_train(self, state, actions, rewards, next_actions, latent_gene, lens, reward_keep=True,
                      attn_seed=0, attn_offset=0, ff_offset=0):
        """Reference-mode (autograd) learn forward; the product learn step is train.FusedTrainStep.
        Dropout masks are the same counter-based streams as the fused step's."""
        c = self.cfg
        b, n, _ = state.shape
        tr = self.transformer
        state_embed = self._lin(state, self.to_state_embed)
        sum_embeds = self.embed_actions(actions) + rewards[..., None] * self.reward_embed * float(reward_keep)
        x = self._lin(state, tr.project_in) + sum_embeds
        H, dh, I = c.heads, c.dim_head, c.inner
        pos = torch.arange(n, device=state.device, dtype=torch.float32)
        inv = tr.attn_layers.rotary_pos_emb.inv_freq
        freqs = (pos[:, None] * inv[None, :]).repeat_interleave(2, dim=-1)
        cos, sin = freqs.cos(), freqs.sin()
        rot = freqs.shape[-1]
        xq = xk = 1.
        if c.rotary_xpos:   # x-transformers RotaryEmbedding(use_xpos): scale ** ((pos - n // 2) / scale_base)
            sc = (torch.arange(0, rot, 2, device=state.device, dtype=torch.float32) + 0.4 * rot) / (1.4 * rot)
            xq = (sc[None, :] ** ((pos - n // 2) / c.xpos_scale_base)[:, None]).repeat_interleave(2, dim=-1)
            xk = xq ** -1.
        scale = c.qk_norm_scale if c.qk_norm else dh ** -0.5
        p_drop = c.dropout if self.training else 0.
        first_v = None
        split = lambda t: t.reshape(b, n, H, dh).permute(0, 2, 1, 3)
        for li, (attn_l, ff_l) in enumerate(self.blocks()):
            (ln_a, _, _), blk, _ = attn_l
            xn = ln_a(x)
            P = self._proj[li]
            # one projection for q | k | v | gate | mix: one well-shaped GEMM, gradient into the flat buffer
            bias = None
            if P['b'] is not None:
                bias = torch.cat((self._zero_bias(3 * I, x), P['b']))
            proj = ops.xlinear(xn, P['w'], bias, P['wg'], P['bg'], self._ws, bg_off=3 * I)
            q, k, v = split(proj[..., :I]), split(proj[..., I:2 * I]), split(proj[..., 2 * I:3 * I])
            gate_pre = proj[..., 3 * I:4 * I] if c.gate_values else None
            orig_v = v
            if P['mix'] and first_v is not None:
                mix = torch.sigmoid(proj[..., -H:]).permute(0, 2, 1)[..., None]
                v = v.lerp(first_v, mix)
            if first_v is None:
                first_v = orig_v
            if c.qk_norm:
                q, k = F.normalize(q, dim=-1), F.normalize(k, dim=-1)
            q = torch.cat((q[..., :rot] * cos * xq + _rotate_half(q[..., :rot]) * sin * xq, q[..., rot:]), dim=-1)
            k = torch.cat((k[..., :rot] * cos * xk + _rotate_half(k[..., :rot]) * sin * xk, k[..., rot:]), dim=-1)
            o = ops.attention(q, k, v, lens, scale, p_drop, attn_seed, attn_offset, li)
            o = o.permute(0, 2, 1, 3).reshape(b, n, I)
            if gate_pre is not None:
                o = o * gate_pre.sigmoid()
            x = self._lin(o, blk.to_out) + x
            (ln_f, _, _), ffb, _ = ff_l
            if c.ff_glu:   # GLU projection, then value * gelu(gate) + dropout (the fused step's mask stream)
                h = ops.glu_drop(self._lin(ln_f(x), ffb.ff[0].proj), p_drop, attn_seed, ff_offset, li)
            else:
                f0 = ffb.ff[0][0]   # Linear + GELU + Dropout in one GEMM epilogue (the fused step's mask stream)
                h = ops.linear_gelu_drop(ln_f(x), f0.weight, f0.bias, f0.weight.grad,
                                         f0.bias.grad if f0.bias is not None else None, self._ws, p_drop,
                                         attn_seed, ff_offset, li)
            x = self._lin(h, ffb.ff[2]) + x
        embed = tr.attn_layers.final_norm(x)
        ewa = torch.cat((embed, self.embed_actions(next_actions)), dim=-1)
        pred_raw = self._lin(F.silu(self._lin(ewa, self.to_pred[0])), self.to_pred[2])
        done_logit = self._lin(ewa, self.to_pred_done[0])[..., 0]
        f = c.frac_head_grad
        embed = embed.detach() * (1. - f) + embed * f
        ac_in = torch.cat((embed, state_embed), dim=-1)
        if c.evolutionary:
            lat = self._lin(latent_gene, self.latent_to_embed)
            ac_in = torch.cat((ac_in, lat[:, None, :].expand(-1, n, -1)), dim=-1)
        hd = self._head1
        hid = F.silu(ops.xlinear(ac_in, hd['w'], hd['b'], hd['wg'], hd['bg'], self._ws))
        d2 = 2 * c.dim
        raw_actions = self._lin(hid[..., :d2], self.action_head[2])
        values = self._lin(hid[..., d2:], self.critic_head[2])
        return raw_actions, values, pred_raw, done_logit
