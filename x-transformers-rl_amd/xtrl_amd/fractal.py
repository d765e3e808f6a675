"""Fractal policy body: FractalEncoder / FractalWorldModelActorCritic forward on the
HIP kernels.

Mirrors x_transformers_rl/fractal_rl.py module-for-module with the reference's parameter names,
so reference checkpoints load with ``load_state_dict`` (e.g. the committed
fractal_experiments/frala_easy_final/final_fractal_agent.pt, read with torch.load(weights_only=True)).
The modules here only hold parameters; ``forward`` runs on libxtrl_hip.so (GEMM with fused bias /
GELU / SiLU / ReLU, bidirectional attention on token-major q/k/v, and the row kernels of
csrc/fractal.hip) and raises without an MI355X — there is no CPU path.

Forward semantics (eval mode: the reference's dropouts are identity at inference):
  FractalProcessingBlock  post-norm  x = LN1(x + SelfAttn(x)); x = LN2(x + CrossAttn(x, g)); x = LN3(x + FF(x))
                          (fractal_rl.py:120-136).  The global state g is ONE token, so the
                          cross-attention softmax is over a single key and equals 1 exactly:
                          CrossAttn(x, g) = W_out W_v g for every query position (computed as two
                          (b x d) GEMMs and broadcast inside the add-LayerNorm kernel).
  FractalEncoder          fractal_rl.py:274-346 — per level: + level embedding, block, global state
                          += Linear(mean_n(level)); output = final_aggregation(cat(mean_n(proj_i(level_i)), g)).
                          The hypernetwork variant's generated weights are unused by the reference
                          (:262-268), so its forward is the base block's.  upscale/downscale layers
                          are built (parameter parity) but unused, as in the reference.
  FractalWorldModelActorCritic  fractal_rl.py:549-619 (frac_gradient is the identity in forward).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F
from torch import nn

from . import _lib as L
from . import ops


def _sinusoidal(levels, dim):
    """FractalLevelEmbedding scale embeddings (fractal_rl.py:50-62)."""
    pos = torch.arange(levels, dtype=torch.float32)[:, None]
    div = torch.exp(torch.arange(0, dim, 2, dtype=torch.float32) * -(math.log(10000.0) / dim))
    emb = torch.zeros(levels, dim)
    emb[:, 0::2] = torch.sin(pos * div)
    emb[:, 1::2] = torch.cos(pos * div)
    return emb


class FractalLevelEmbedding(nn.Module):
    def __init__(self, embed_dim, max_levels=8):
        super().__init__()
        self.level_embeds = nn.Parameter(torch.randn(max_levels, embed_dim) * 0.02)
        self.register_buffer('scale_embeds', _sinusoidal(max_levels, embed_dim))


class Attention(nn.Module):
    """x-transformers Attention parameter layout (no bias projections)."""

    def __init__(self, dim, heads, dim_head):
        super().__init__()
        inner = heads * dim_head
        self.heads, self.dim_head = heads, dim_head
        self.to_q = nn.Linear(dim, inner, bias=False)
        self.to_k = nn.Linear(dim, inner, bias=False)
        self.to_v = nn.Linear(dim, inner, bias=False)
        self.to_out = nn.Linear(inner, dim, bias=False)


class FeedForward(nn.Module):
    """x-transformers FeedForward layout: ff.0.0 Linear(d, mult d) + GELU, ff.1 Dropout, ff.2 Linear."""

    def __init__(self, dim, mult=4, dropout=0.):
        super().__init__()
        self.ff = nn.Sequential(nn.Sequential(nn.Linear(dim, dim * mult), nn.GELU()), nn.Dropout(dropout),
                                nn.Linear(dim * mult, dim))


class FractalProcessingBlock(nn.Module):
    def __init__(self, dim, heads=8, dim_head=64, ff_mult=4, dropout=0.1):
        super().__init__()
        self.self_attn = Attention(dim, heads, dim_head)
        self.global_attn = Attention(dim, heads, dim_head)
        self.ff = FeedForward(dim, ff_mult, dropout)
        self.norm1, self.norm2, self.norm3 = nn.LayerNorm(dim), nn.LayerNorm(dim), nn.LayerNorm(dim)


def _add_ln(x, r, r_rep, norm, out):
    """out = norm(x + r[row // r_rep]) (nn.LayerNorm with its own eps / weight / bias)."""
    L.check(L.lib().xtrl_add_layernorm(L.ptr(x), x.stride(0), L.ptr(r), r.stride(0), r_rep, L.ptr(norm.weight),
                                       L.ptr(norm.bias), L.ptr(out), out.stride(0), x.shape[0], x.shape[1],
                                       float(norm.eps), L.stream()), 'add_layernorm')


class _Buffers:
    """Per-call device scratch (token-major activations)."""

    def __init__(self, b, n, d, heads, inner, ff, dev):
        T = b * n
        e = lambda *s: torch.empty(*s, device=dev, dtype=torch.float32)
        self.qkv, self.o, self.a, self.lse = e(T, 3 * inner), e(T, inner), e(T, d), e(b * heads * n)
        self.x1, self.x2, self.h, self.f = e(T, d), e(T, d), e(T, ff), e(T, d)
        self.c1, self.c2, self.mean = e(b, inner), e(b, d), e(b, d)


class FractalEncoder(nn.Module):
    def __init__(self, input_dim, embed_dim=512, num_levels=4, heads=8, dim_head=64, ff_mult=4, dropout=0.1,
                 global_state_dim=None, share_weights=False, use_hypernetwork=False):
        super().__init__()
        self.embed_dim, self.num_levels, self.heads, self.dim_head = embed_dim, num_levels, heads, dim_head
        self.ff_mult = ff_mult
        self.share_weights, self.use_hypernetwork = share_weights, use_hypernetwork
        self.global_state_dim = global_state_dim or embed_dim
        assert self.global_state_dim == embed_dim, 'the global state is read by attention over embed_dim tokens'
        self.input_embed = nn.Linear(input_dim, embed_dim)
        self.level_embedding = FractalLevelEmbedding(embed_dim, num_levels)
        self.global_state_init = nn.Parameter(torch.randn(1, 1, self.global_state_dim) * 0.02)
        self.global_state_update = nn.Linear(embed_dim, self.global_state_dim)
        blk = lambda: FractalProcessingBlock(embed_dim, heads, dim_head, ff_mult, dropout)
        if share_weights:
            self.fractal_block = blk()
        elif use_hypernetwork:
            self.hypernet = nn.Sequential(nn.Linear(embed_dim, embed_dim * 2), nn.ReLU(),
                                          nn.Linear(embed_dim * 2, embed_dim))
            self.base_block = blk()
        else:
            self.fractal_blocks = nn.ModuleList([blk() for _ in range(num_levels)])
        self.upscale_layers = nn.ModuleList([nn.Linear(embed_dim, embed_dim) for _ in range(num_levels - 1)])
        self.downscale_layers = nn.ModuleList([nn.Linear(embed_dim, embed_dim) for _ in range(num_levels - 1)])
        self.level_projections = nn.ModuleList([nn.Linear(embed_dim, embed_dim) for _ in range(num_levels)])
        self.final_aggregation = nn.Sequential(nn.Linear(embed_dim * (num_levels + 1), embed_dim * 2), nn.ReLU(),
                                               nn.Linear(embed_dim * 2, embed_dim))

    def get_fractal_block(self, level_idx):
        if self.share_weights:
            return self.fractal_block
        if self.use_hypernetwork:
            return self.base_block
        return self.fractal_blocks[level_idx]

    # -- HIP forward ------------------------------------------------------------------------------
    def _block(self, blk, x, g, lens, b, n, buf, out):
        lib, s = L.lib(), L.stream()
        d, H, dh = self.embed_dim, self.heads, self.dim_head
        I = H * dh
        sa, ga = blk.self_attn, blk.global_attn
        for j, lin in enumerate((sa.to_q, sa.to_k, sa.to_v)):
            ops.gemm(x, lin.weight, out=buf.qkv[:, j * I:(j + 1) * I])
        q = buf.qkv
        L.check(lib.xtrl_attn_fwd_tokens(L.ptr(q), 3 * I, L.ptr(q[:, I:]), 3 * I, L.ptr(q[:, 2 * I:]), 3 * I,
                                         L.ptr(lens), L.ptr(buf.o), I, L.ptr(buf.lse), b, H, n, dh,
                                         1.0 / math.sqrt(dh), 0, s), 'attn_fwd_tokens')
        ops.gemm(buf.o, sa.to_out.weight, out=buf.a)
        _add_ln(x, buf.a, 1, blk.norm1, buf.x1)
        # cross-attention to the one-token global state: softmax over one key == 1
        ops.gemm(g, ga.to_v.weight, out=buf.c1)
        ops.gemm(buf.c1, ga.to_out.weight, out=buf.c2)
        _add_ln(buf.x1, buf.c2, n, blk.norm2, buf.x2)
        ff0, ff2 = blk.ff.ff[0][0], blk.ff.ff[2]
        ops.gemm(buf.x2, ff0.weight, ff0.bias, act=L.ACT_GELU, out=buf.h)
        ops.gemm(buf.h, ff2.weight, ff2.bias, out=buf.f)
        _add_ln(buf.x2, buf.f, 1, blk.norm3, out)

    def forward(self, x, mask=None, return_all_levels=False, out=None):
        """x [b, n, input_dim] -> aggregated [b, embed_dim] (and the level outputs [b, n, embed_dim]).
        mask [b, n] bool: key-padding mask, prefix form (keys j < len_b)."""
        lib, s = L.lib(), L.stream()
        if x.ndim == 2:
            x = x[:, None]
        b, n, _ = x.shape
        d, I, Lv = self.embed_dim, self.heads * self.dim_head, self.num_levels
        dev = x.device
        x2 = x.reshape(b * n, -1).float().contiguous()
        if mask is None:
            lens = torch.full((b,), n, dtype=torch.int32, device=dev)
        else:
            lens = mask.sum(-1).to(torch.int32)
            assert bool((mask == (torch.arange(n, device=dev)[None] < lens[:, None].long())).all()), \
                'key-padding masks must be prefix masks'
        buf = _Buffers(b, n, d, self.heads, I, d * self.ff_mult, dev)
        cur = ops.gemm(x2, self.input_embed.weight, self.input_embed.bias)
        g = torch.empty(b, d, device=dev)
        L.check(lib.xtrl_rows_add(None, 0, L.ptr(self.global_state_init.reshape(-1)), L.ptr(g), d, b, d, s),
                'rows_add')
        emb = torch.empty(Lv, d, device=dev)
        le = self.level_embedding
        for li in range(Lv):   # level embeds + scale embeds, row by row (scale_embeds rows differ per level)
            L.check(lib.xtrl_rows_add(L.ptr(le.level_embeds[li]), d, L.ptr(le.scale_embeds[li]), L.ptr(emb[li]), d,
                                      1, d, s), 'rows_add')
        levels = []
        allf = torch.empty(b, (Lv + 1) * d, device=dev)
        for li in range(Lv):
            feats = torch.empty(b * n, d, device=dev)
            L.check(lib.xtrl_rows_add(L.ptr(cur), d, L.ptr(emb[li]), L.ptr(feats), d, b * n, d, s), 'rows_add')
            outl = torch.empty(b * n, d, device=dev)
            self._block(self.get_fractal_block(li), feats, g, lens, b, n, buf, outl)
            L.check(lib.xtrl_seq_mean(L.ptr(outl), d, b, n, d, L.ptr(buf.mean), d, s), 'seq_mean')
            ops.gemm(buf.mean, self.global_state_update.weight, self.global_state_update.bias, residual=g, out=g)
            levels.append(outl)
            cur = outl
        for i, lv in enumerate(levels):
            pj = self.level_projections[i]
            p = ops.gemm(lv, pj.weight, pj.bias, out=buf.f)
            L.check(lib.xtrl_seq_mean(L.ptr(p), d, b, n, d, L.ptr(allf[:, i * d:]), (Lv + 1) * d, s), 'seq_mean')
        L.check(lib.xtrl_seq_mean(L.ptr(g), d, b, 1, d, L.ptr(allf[:, Lv * d:]), (Lv + 1) * d, s), 'seq_mean')
        fa0, fa2 = self.final_aggregation[0], self.final_aggregation[2]
        hid = ops.gemm(allf, fa0.weight, fa0.bias, act=L.ACT_RELU)
        agg = ops.gemm(hid, fa2.weight, fa2.bias, out=out)
        if return_all_levels:
            return agg, [lv.view(b, n, d) for lv in levels]
        return agg


class SafeEmbedding(nn.Module):
    """x_transformers_rl.py:181-195 layout (embed.weight)."""

    def __init__(self, num_embeds, dim):
        super().__init__()
        self.embed = nn.Embedding(num_embeds, dim)


class FractalWorldModelActorCritic(nn.Module):
    def __init__(self, state_dim, num_actions, critic_dim_pred, critic_min_max_value, embed_dim=512,
                 num_fractal_levels=4, heads=8, dim_head=64, ff_mult=4, dropout=0.1, continuous_actions=False,
                 squash_continuous=False, frac_actor_critic_head_gradient=0.5, entropy_weight=0.02,
                 reward_dropout=0.5, eps_clip=0.2, value_clip=0.4, evolutionary=False, dim_latent_gene=None,
                 normalize_advantages=True, fractal_share_weights=False, fractal_use_hypernetwork=False):
        super().__init__()
        self.state_dim, self.num_actions, self.embed_dim = state_dim, num_actions, embed_dim
        self.continuous, self.evolutionary = continuous_actions, evolutionary
        self.critic_min_max_value = critic_min_max_value
        self.fractal_encoder = FractalEncoder(state_dim, embed_dim, num_fractal_levels, heads, dim_head, ff_mult,
                                              dropout, share_weights=fractal_share_weights,
                                              use_hypernetwork=fractal_use_hypernetwork)
        self.reward_embed = nn.Parameter(torch.ones(embed_dim) * 1e-2)
        self.action_embeds = (nn.Linear(num_actions, embed_dim) if continuous_actions
                              else SafeEmbedding(num_actions, embed_dim))
        self.to_state_embed = nn.Linear(state_dim, embed_dim)
        self.to_pred_done = nn.Sequential(nn.Linear(embed_dim * 2, 1))   # + sigmoid (in xtrl_wm_post)
        self.to_pred = nn.Sequential(nn.Linear(embed_dim * 2, embed_dim), nn.SiLU(),
                                     nn.Linear(embed_dim, 2 * (state_dim + 1)))
        if evolutionary:
            assert dim_latent_gene is not None
            self.latent_to_embed = nn.Linear(dim_latent_gene, embed_dim)
        ac_in = embed_dim * (3 if evolutionary else 2)
        self.critic_head = nn.Sequential(nn.Linear(ac_in, embed_dim * 2), nn.SiLU(),
                                         nn.Linear(embed_dim * 2, critic_dim_pred))
        self.action_head = nn.Sequential(nn.Linear(ac_in, embed_dim * 2), nn.SiLU(),
                                         nn.Linear(embed_dim * 2, num_actions * (2 if continuous_actions else 1)))

    def forward(self, state, actions=None, rewards=None, next_actions=None, latent_gene=None, **kwargs):
        """-> (raw_actions [b, A], values [b, B], state_pred [2, b, S+1] | None, dones [b] | None, cache)."""
        lib, s = L.lib(), L.stream()
        if state.ndim == 2:
            state = state[:, None]
        b, n, S = state.shape
        d, dev = self.embed_dim, state.device
        ac = torch.empty(b, d * (3 if self.evolutionary else 2), device=dev)
        feats, levels = self.fractal_encoder(state, return_all_levels=True, out=ac[:, :d])
        st = state.reshape(b * n, S).float().contiguous()
        se = ops.gemm(st, self.to_state_embed.weight, self.to_state_embed.bias)
        L.check(lib.xtrl_seq_mean(L.ptr(se), d, b, n, d, L.ptr(ac[:, d:]), ac.stride(0), s), 'seq_mean')
        state_pred = dones = None
        if next_actions is not None:
            ewa = torch.empty(b, 2 * d, device=dev)
            L.check(lib.xtrl_seq_mean(L.ptr(ac), ac.stride(0), b, 1, d, L.ptr(ewa), 2 * d, s), 'seq_mean')
            if self.continuous:
                ops.gemm(next_actions.float().contiguous(), self.action_embeds.weight, self.action_embeds.bias,
                         out=ewa[:, d:])
            else:
                na = next_actions.to(torch.int32).contiguous()
                L.check(lib.xtrl_safe_embed(L.ptr(na), b, L.ptr(self.action_embeds.embed.weight), d,
                                            L.ptr(ewa[:, d:]), 2 * d, s), 'safe_embed')
            p0, p2 = self.to_pred[0], self.to_pred[2]
            raw = ops.gemm(ops.gemm(ewa, p0.weight, p0.bias, act=L.ACT_SILU), p2.weight, p2.bias)
            dl = ops.gemm(ewa, self.to_pred_done[0].weight, self.to_pred_done[0].bias)
            state_pred = torch.empty(2, b, S + 1, device=dev)
            dones = torch.empty(b, device=dev)
            L.check(lib.xtrl_wm_post(L.ptr(raw), raw.stride(0), b, S + 1, L.ptr(state_pred), L.ptr(dl), 1,
                                     L.ptr(dones), s), 'wm_post')
        if self.evolutionary and latent_gene is not None:
            ops.gemm(latent_gene.float().contiguous(), self.latent_to_embed.weight, self.latent_to_embed.bias,
                     out=ac[:, 2 * d:])
        a0, a2 = self.action_head[0], self.action_head[2]
        c0, c2 = self.critic_head[0], self.critic_head[2]
        raw_actions = ops.gemm(ops.gemm(ac, a0.weight, a0.bias, act=L.ACT_SILU), a2.weight, a2.bias)
        values = ops.gemm(ops.gemm(ac, c0.weight, c0.bias, act=L.ACT_SILU), c2.weight, c2.bias)
        level_feats = []
        for lv in levels:
            m = torch.empty(b, d, device=dev)
            L.check(lib.xtrl_seq_mean(L.ptr(lv), d, b, n, d, L.ptr(m), d, s), 'seq_mean')
            level_feats.append(m)
        cache = dict(fractal_levels=levels, global_state=None, level_features=level_feats)
        return raw_actions, values, state_pred, dones, cache


# ----------------------------------------------------------------------------------------------
# Per-timestep, causal fractal policy body: the FractalWorldModelActorCritic of
# fractal_rl.py:349-619 with every sequence pooling made causal, so position t sees states 0..t
# only and the body stands in for the Decoder inside the Learner (PPO / world-model losses per
# timestep, KV-cached rollout).  Decision log:
#   * self-attention causal + key padding (the reference's encoder attends bidirectionally);
#   * the global state is per timestep: g_t <- g_t + W_gu mean_{s <= t}(level_s) + b_gu
#     (reference: one state per sequence from mean_n);
#   * cross-attention reads g_t (one key, softmax == 1: W_out W_v g_t);
#   * level outputs pooled causally: p_l,t = W_p,l mean_{s <= t}(level_s) + b_p,l (the projection of
#     the running mean == the running mean of the projections);
#   * features_t = final_aggregation([p_0,t | ... | g_t]); heads per timestep on
#     [frac_gradient(features_t) | to_state_embed(s_t) (| latent)] (reference: state embed mean-pooled);
#   * like the reference forward, the encoder reads the states only (the action / reward arguments
#     condition nothing but the world-model heads' next action).
# Parameter names are the reference class's, so its checkpoints load.
# ----------------------------------------------------------------------------------------------


class FractalPolicyActorCritic(FractalWorldModelActorCritic):
    def __init__(self, c, levels):
        super().__init__(c.state_dim, c.num_actions, c.num_bins, c.reward_range, embed_dim=c.dim,
                         num_fractal_levels=levels, heads=c.heads, dim_head=c.dim_head, ff_mult=c.ff_mult,
                         dropout=c.dropout, continuous_actions=c.continuous, squash_continuous=c.squash,
                         evolutionary=c.evolutionary, dim_latent_gene=c.dim_gene if c.evolutionary else None)
        self.cfg, self.levels = c, levels
        lo, hi = c.reward_range
        support = torch.linspace(lo, hi, c.num_bins + 1, dtype=torch.float32)
        self.register_buffer('hl_support', support, persistent=False)
        self.register_buffer('hl_centers', (support[:-1] + support[1:]) / 2, persistent=False)
        self.hl_sigma = c.hl_sigma_ratio * (hi - lo) / c.num_bins

    def hl_value(self, logits):
        return (logits.softmax(dim=-1) * self.hl_centers).sum(-1)

    def block_prefix(self, li):
        """Parameter-name prefix of the block level ``li`` runs (FractalEncoder.get_fractal_block)."""
        enc = self.fractal_encoder
        if enc.share_weights:
            return 'fractal_encoder.fractal_block.'
        if enc.use_hypernetwork:
            return 'fractal_encoder.base_block.'
        return f'fractal_encoder.fractal_blocks.{li}.'

    def flat_buckets_names(self):
        """Parameter groups of the flat buffer, bucketed in the order the fused fractal backward
        completes them (csrc/train.hip fractal_train_backward records an event pair per bucket for the
        overlapped data-parallel all-reduce): [heads, action embedding, final aggregation], [level L-1's
        block + level projection], ..., [level 0's], [input embedding, global-state init / update,
        level embeddings (accumulated over every level) and the parameters no forward reads].  A shared
        (share_weights / hypernetwork) block accumulates over the levels, so it goes to the last bucket.
        Weights used as one GEMM operand are adjacent groups: each block's to_q | to_k | to_v, the
        actor | critic first layers, to_pred.0 | to_pred_done.0 (weights and biases); groups whose size
        is not a multiple of 4 floats move to the last bucket, so every GEMM weight starts 16-byte
        aligned.  -> list of buckets, each a list of groups."""
        params = dict(self.named_parameters())
        taken = set()

        def grp(names):
            taken.update(names)
            return list(names)

        def under(*prefixes):
            return [grp([n]) for n in params if n not in taken and n.startswith(prefixes)]

        enc = self.fractal_encoder
        heads = [grp(['action_head.0.weight', 'critic_head.0.weight']), grp(['action_head.0.bias', 'critic_head.0.bias']),
                 grp(['to_pred.0.weight', 'to_pred_done.0.weight']), grp(['to_pred.0.bias', 'to_pred_done.0.bias'])]
        heads += under('action_head.', 'critic_head.', 'to_pred.', 'to_pred_done.', 'to_state_embed.',
                       'latent_to_embed.', 'action_embeds.', 'fractal_encoder.final_aggregation.')
        per_level = not (enc.share_weights or enc.use_hypernetwork)
        levels = []
        for li in reversed(range(self.levels)):
            g = []
            if per_level:
                pre = self.block_prefix(li)
                g.append(grp([pre + 'self_attn.to_q.weight', pre + 'self_attn.to_k.weight', pre + 'self_attn.to_v.weight']))
                g += under(pre + 'norm3.', pre + 'ff.', pre + 'norm2.', pre + 'norm1.', pre + 'global_attn.to_out.',
                           pre + 'global_attn.to_v.', pre + 'self_attn.to_out.')
            g += under(f'fractal_encoder.level_projections.{li}.')
            levels.append(g)
        if not per_level:
            pre = self.block_prefix(0) + 'self_attn.'
            tail0 = [grp([pre + 'to_q.weight', pre + 'to_k.weight', pre + 'to_v.weight'])]
        else:
            tail0 = []
        tail = tail0 + [grp([n]) for n in params if n not in taken]
        buckets = [heads] + levels + [tail]
        size = lambda g: sum(params[n].numel() for n in g)
        odd = [g for b in buckets for g in b if size(g) % 4]
        buckets = [[g for g in b if size(g) % 4 == 0] for b in buckets]
        buckets[-1] += odd
        return buckets

    def flat_order(self):
        """Every parameter once, in bucket order (flat_buckets_names)."""
        return [n for b in self.flat_buckets_names() for g in b for n in g]

    def flat_bucket_ranges(self, flat):
        from .model import bucket_ranges
        return bucket_ranges(self.flat_buckets_names(), flat)

    def bind_flat(self, flat, ws):
        self._flat, self._ws = flat, ws

    def embed_actions(self, actions):
        if self.cfg.continuous:
            return self._lin(actions, self.action_embeds)
        onehot = F.one_hot(actions.clamp(min=0), self.cfg.num_actions).to(torch.float32)
        onehot = onehot * (actions >= 0)[..., None].to(torch.float32)
        return onehot @ self.action_embeds.embed.weight

    def _lin(self, x, mod):
        b = mod.bias
        return ops.xlinear(x, mod.weight, b, mod.weight.grad, b.grad if b is not None else None, self._ws)

    def level_embed(self, li):
        le = self.fractal_encoder.level_embedding
        return le.level_embeds[li] + le.scale_embeds[li]

    def forward_train(self, state, actions, rewards, next_actions, latent_gene, lens, reward_keep=True,
                      attn_seed=0, attn_offset=0, ff_offset=0):
        """Learn-step forward (autograd over the HIP GEMM / flash-attention ops; LayerNorm, running
        means and concatenations as PyTorch ops) -> (raw_actions, values, pred_raw, done_logit)."""
        c = self.cfg
        enc = self.fractal_encoder
        b, n, _ = state.shape
        d, H, dh = c.dim, c.heads, c.dim_head
        I = H * dh
        p_drop = c.dropout if self.training else 0.
        split = lambda t: t.reshape(b, n, H, dh).permute(0, 2, 1, 3)
        cnt = torch.arange(1, n + 1, device=state.device, dtype=torch.float32)[None, :, None]
        x = self._lin(state, enc.input_embed)
        g = enc.global_state_init.reshape(1, 1, d).expand(b, n, d)
        projs = []
        for li in range(self.levels):
            blk = enc.get_fractal_block(li)
            x = x + self.level_embed(li)
            sa, ga = blk.self_attn, blk.global_attn
            q, k, v = split(self._lin(x, sa.to_q)), split(self._lin(x, sa.to_k)), split(self._lin(x, sa.to_v))
            o = ops.attention(q.contiguous(), k.contiguous(), v.contiguous(), lens, dh ** -0.5, p_drop, attn_seed,
                              attn_offset, li)
            o = o.permute(0, 2, 1, 3).reshape(b, n, I)
            x1 = blk.norm1(x + self._lin(o, sa.to_out))
            x2 = blk.norm2(x1 + self._lin(self._lin(g, ga.to_v), ga.to_out))
            ff0, ff2 = blk.ff.ff[0][0], blk.ff.ff[2]
            h = ops.linear_gelu_drop(x2, ff0.weight, ff0.bias, ff0.weight.grad, ff0.bias.grad, self._ws, p_drop,
                                     attn_seed, ff_offset, li)   # Linear + GELU + Dropout in one epilogue
            x3 = blk.norm3(x2 + self._lin(h, ff2))
            mean = x3.cumsum(dim=1) / cnt
            projs.append(self._lin(mean, enc.level_projections[li]))
            g = g + self._lin(mean, enc.global_state_update)
            x = x3
        fa0, fa2 = enc.final_aggregation[0], enc.final_aggregation[2]
        feat = self._lin(F.relu(self._lin(torch.cat(projs + [g], dim=-1), fa0)), fa2)
        ewa = torch.cat((feat, self.embed_actions(next_actions)), dim=-1)
        pred_raw = self._lin(F.silu(self._lin(ewa, self.to_pred[0])), self.to_pred[2])
        done_logit = self._lin(ewa, self.to_pred_done[0])[..., 0]
        f = c.frac_head_grad
        feat = feat.detach() * (1. - f) + feat * f
        ac_in = torch.cat((feat, self._lin(state, self.to_state_embed)), dim=-1)
        if c.evolutionary:
            lat = self._lin(latent_gene, self.latent_to_embed)
            ac_in = torch.cat((ac_in, lat[:, None, :].expand(-1, n, -1)), dim=-1)
        raw_actions = self._lin(F.silu(self._lin(ac_in, self.action_head[0])), self.action_head[2])
        values = self._lin(F.silu(self._lin(ac_in, self.critic_head[0])), self.critic_head[2])
        return raw_actions, values, pred_raw, done_logit
