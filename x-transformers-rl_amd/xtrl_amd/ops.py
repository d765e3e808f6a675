"""Torch-facing wrappers of the HIP kernels (autograd Functions for the learn step).

Every op checks shapes on the host before launching (the kernels assume them) and runs on the
current torch stream.  No op has a CPU implementation."""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib as L


def _f32c(t):
    assert t.dtype == torch.float32 and t.is_cuda and t.is_contiguous(), (t.dtype, t.device, t.shape)
    return t


# --------------------------------------------------------------------------------------------
# GEMM / LayerNorm
# --------------------------------------------------------------------------------------------


def gemm(x, w, bias=None, ln_gamma=None, residual=None, act=L.ACT_NONE, out=None):
    """act(LN?(x) @ w.T + bias) (+ residual) on the f32 MFMA path.  x [M, K] (row stride may
    exceed K), w [N, K] contiguous."""
    lib = L.lib()
    M, K = x.shape
    N = w.shape[0]
    assert w.shape[1] == K and x.stride(1) == 1 and w.is_contiguous()
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=torch.float32)
    if bias is not None:
        assert bias.shape == (N,) and bias.is_contiguous()
    if ln_gamma is not None:
        assert ln_gamma.shape == (K,)
    if residual is not None:
        assert residual.shape == (M, N) and residual.stride(1) == 1
    L.check(lib.xtrl_gemm_f32(L.ptr(x), x.stride(0), L.ptr(w), K, L.ptr(bias), L.ptr(ln_gamma), L.ptr(residual),
                              residual.stride(0) if residual is not None else 0, L.ptr(out), out.stride(0), None, 0,
                              M, N, K, act, L.stream()), 'gemm')
    return out


def gemm_ex(a, b, trans_a, trans_b, M, N, K, out, bias=None, beta=0.):
    """C[M, N] = beta C + A . B (+ bias); operand layouts as in include/xtrl_hip.h (xtrl_gemm_ex)."""
    L.check(L.lib().xtrl_gemm_ex(int(trans_a), int(trans_b), L.ptr(a), a.stride(0), L.ptr(b), b.stride(0), L.ptr(bias),
                                 L.ptr(out), out.stride(0), M, N, K, float(beta), L.stream()), 'gemm_ex')
    return out


def wgrad(dy, x, dw, ws, beta=1.):
    """dw[N, K] = beta dw + dy[M, N]^T x[M, K]  (split over the M tokens, deterministic)."""
    M, N = dy.shape
    K = x.shape[1]
    assert dw.shape == (N, K) and dw.is_contiguous() and x.stride(1) == 1 and dy.stride(1) == 1
    L.check(L.lib().xtrl_gemm_wgrad(L.ptr(dy), dy.stride(0), L.ptr(x), x.stride(0), L.ptr(dw), K, M, N, K,
                                    float(beta), L.ptr(ws), ws.numel(), L.stream()), 'gemm_wgrad')


class XLinearFn(torch.autograd.Function):
    """nn.Linear on the library GEMMs (the reference-mode learn step; the fractal policy body's
    product path): forward y = x W^T + b and input gradient dx = dy W on gemm_run (split-bf16
    products on the large-tile geometry), the weight gradient by the split-K HIP GEMM with the bias
    gradient folded into it, both accumulated straight into the flat gradient buffer (no
    per-parameter accumulation pass, no separate column-sum launch)."""

    @staticmethod
    def forward(ctx, x, w, b, wg, bg, bg_off, ws):
        K = x.shape[-1]
        N = w.shape[0]
        x2 = x.reshape(-1, K)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        M = x2.shape[0]
        assert w.is_contiguous() and (b is None or b.is_contiguous())
        y = torch.empty(M, N, device=x.device, dtype=torch.float32)
        if M:
            gemm_ex(x2, w, 0, 0, M, N, K, y, bias=b)
        ctx.save_for_backward(x2, w)
        ctx.extra = (wg, bg, bg_off, ws, x.shape)
        return y.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        wg, bg, bg_off, ws, xshape = ctx.extra
        N, K = w.shape
        dy2 = dy.reshape(-1, N)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        M = dy2.shape[0]
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, K, device=dy.device, dtype=torch.float32)
            if M:
                gemm_ex(dy2, w, 0, 1, M, K, N, dx)
            dx = dx.view(xshape)
        if wg is not None and M:
            L.check(L.lib().xtrl_gemm_wgrad_db(L.ptr(dy2), dy2.stride(0), L.ptr(x2), x2.stride(0), L.ptr(wg), K, M, N,
                                               K, 1., L.ptr(ws), ws.numel(), L.ptr(bg), int(bg_off), L.stream()),
                    'gemm_wgrad_db')
        elif bg is not None:
            bg.add_(dy2[:, bg_off:].sum(0))
        return dx, None, None, None, None, None, None


def xlinear(x, w, b, wg, bg, ws, bg_off=0):
    return XLinearFn.apply(x, w, b, wg, bg, bg_off, ws)


class LinearGeluDropFn(torch.autograd.Function):
    """h = drop(gelu(x W^T + b)) in one GEMM epilogue that also saves drop(gelu'(.)) (the feed-forward
    first Linear + GELU + Dropout); backward: one multiply by the saved derivative, then the linear
    backward of XLinearFn.  The dropout keep bits are the xtrl_ff_dropout_mask / fused-step stream."""

    @staticmethod
    def forward(ctx, x, w, b, wg, bg, ws, p, seed, offset, layer):
        K = x.shape[-1]
        N = w.shape[0]
        x2 = x.reshape(-1, K)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        M = x2.shape[0]
        assert w.is_contiguous() and (b is None or b.is_contiguous())
        y = torch.empty(M, N, device=x.device, dtype=torch.float32)
        deriv = torch.empty(M, N, device=x.device, dtype=torch.float32)
        L.check(L.lib().xtrl_linear_gelu_drop(L.ptr(x2), K, L.ptr(w), L.ptr(b), L.ptr(y), N, L.ptr(deriv), N, M, N, K,
                                              float(p), int(seed) & (2 ** 64 - 1), int(offset) & 0xFFFFFFFF,
                                              int(layer), L.stream()), 'linear_gelu_drop')
        ctx.save_for_backward(x2, w, deriv)
        ctx.extra = (wg, bg, ws, x.shape)
        return y.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dh):
        x2, w, deriv = ctx.saved_tensors
        wg, bg, ws, xshape = ctx.extra
        N, K = w.shape
        g = (dh.reshape(-1, N) * deriv).contiguous()
        M = g.shape[0]
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, K, device=g.device, dtype=torch.float32)
            if M:
                gemm_ex(g, w, 0, 1, M, K, N, dx)
            dx = dx.view(xshape)
        if wg is not None and M:
            L.check(L.lib().xtrl_gemm_wgrad_db(L.ptr(g), N, L.ptr(x2), K, L.ptr(wg), K, M, N, K, 1., L.ptr(ws), ws.numel(),
                                               L.ptr(bg), 0, L.stream()), 'gemm_wgrad_db')
        elif bg is not None:
            bg.add_(g.sum(0))
        return dx, None, None, None, None, None, None, None, None, None


def linear_gelu_drop(x, w, b, wg, bg, ws, p, seed, offset, layer):
    return LinearGeluDropFn.apply(x, w, b, wg, bg, ws, p, seed, offset, layer)


class GluDropFn(torch.autograd.Function):
    """x-transformers GLU project-in after its projection + the feed-forward dropout (world_model
    ['ff_glu']): u [.., 2 ff] = [value | gate] -> h = drop(value * gelu(gate)) [.., ff]; keep bits of the
    xtrl_ff_dropout_mask / fused-step stream (xtrl_glu_drop_fwd / _bwd)."""

    @staticmethod
    def forward(ctx, u, p, seed, offset, layer):
        F2 = u.shape[-1]
        assert F2 % 2 == 0
        ff = F2 // 2
        u2 = _f32c(u.reshape(-1, F2).contiguous())
        M = u2.shape[0]
        h = torch.empty(M, ff, device=u.device, dtype=torch.float32)
        args = (float(p), int(seed) & (2 ** 64 - 1), int(offset) & 0xFFFFFFFF, int(layer))
        L.check(L.lib().xtrl_glu_drop_fwd(L.ptr(u2), F2, L.ptr(h), ff, M, ff, *args, L.stream()), 'glu_drop_fwd')
        ctx.save_for_backward(u2)
        ctx.extra = (args, u.shape)
        return h.view(*u.shape[:-1], ff)

    @staticmethod
    def backward(ctx, dh):
        (u2,) = ctx.saved_tensors
        args, ushape = ctx.extra
        M, F2 = u2.shape
        ff = F2 // 2
        dh2 = dh.reshape(-1, ff).contiguous()
        du = torch.empty(M, F2, device=dh.device, dtype=torch.float32)
        L.check(L.lib().xtrl_glu_drop_bwd(L.ptr(dh2), ff, L.ptr(u2), F2, L.ptr(du), F2, M, ff, *args, L.stream()),
                'glu_drop_bwd')
        return du.view(ushape), None, None, None, None


def glu_drop(u, p, seed, offset, layer):
    return GluDropFn.apply(u, p, seed, offset, layer)


def layernorm(x, gamma, out=None):
    lib = L.lib()
    M, D = x.shape
    if out is None:
        out = torch.empty(M, D, device=x.device, dtype=torch.float32)
    L.check(lib.xtrl_layernorm_f32(L.ptr(x), x.stride(0), L.ptr(gamma), L.ptr(out), out.stride(0), M, D,
                                   L.stream()), 'layernorm')
    return out


# --------------------------------------------------------------------------------------------
# training attention
# --------------------------------------------------------------------------------------------


class AttentionFn(torch.autograd.Function):
    """softmax(q k^T * scale + causal/key-padding mask) with post-softmax dropout, times v."""

    @staticmethod
    def forward(ctx, q, k, v, lens, scale, dropout_p, seed, offset, sub):
        lib = L.lib()
        b, H, n, dh = q.shape
        for t in (q, k, v):
            _f32c(t)
            assert t.shape == (b, H, n, dh)
        assert lens.dtype == torch.int32 and lens.shape == (b,)
        o = torch.empty_like(q)
        lse = torch.empty(b, H, n, device=q.device, dtype=torch.float32)
        L.check(lib.xtrl_attn_fwd(L.ptr(q), L.ptr(k), L.ptr(v), L.ptr(lens), L.ptr(o), L.ptr(lse), b, H, n, dh,
                                  float(scale), float(dropout_p), int(seed), int(offset), int(sub), L.stream()),
                'attn_fwd')
        ctx.save_for_backward(q, k, v, lens, o, lse)
        ctx.cfg = (float(scale), float(dropout_p), int(seed), int(offset), int(sub))
        return o

    @staticmethod
    def backward(ctx, do):
        lib = L.lib()
        q, k, v, lens, o, lse = ctx.saved_tensors
        scale, p, seed, offset, sub = ctx.cfg
        b, H, n, dh = q.shape
        do = do.contiguous()
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        delta = torch.empty(b, H, n, device=q.device, dtype=torch.float32)
        L.check(lib.xtrl_attn_bwd(L.ptr(q), L.ptr(k), L.ptr(v), L.ptr(lens), L.ptr(o), L.ptr(lse), L.ptr(do),
                                  L.ptr(dq), L.ptr(dk), L.ptr(dv), L.ptr(delta), b, H, n, dh, scale, p, seed, offset,
                                  sub, L.stream()), 'attn_bwd')
        return dq, dk, dv, None, None, None, None, None, None


def attention(q, k, v, lens, scale, dropout_p=0., seed=0, offset=0, sub=0):
    """``offset`` / ``sub``: the dropout stream (Philox c2 base and c3 sub-index = decoder layer)."""
    return AttentionFn.apply(q.contiguous(), k.contiguous(), v.contiguous(), lens, scale, dropout_p, seed, offset,
                             sub)


# --------------------------------------------------------------------------------------------
# fused PPO / critic / world-model / done loss
# --------------------------------------------------------------------------------------------


class LossConsts:
    """Per-minibatch constant tensors + hyper-parameters of the fused loss."""

    def __init__(self, *, actions, old_logp, returns, old_values, dones, lens, real, support, centers, continuous,
                 squash, hl_mean, eps_clip, value_clip, entropy_weight, w_actor, w_critic, w_autoreg, lo, hi, sigma):
        self.__dict__.update(locals())
        del self.__dict__['self']


class LossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, raw_actions, values, pred_raw, done_logit, K: LossConsts):
        lib = L.lib()
        b, n, B = values.shape
        S1 = K.real.shape[-1]
        A = K.old_logp.shape[-1] if K.continuous else raw_actions.shape[-1]
        raw_actions, values, pred_raw, done_logit = (t.contiguous() for t in (raw_actions, values, pred_raw, done_logit))
        assert pred_raw.shape == (b, n, 2 * S1) and done_logit.shape == (b, n)
        assert raw_actions.shape == (b, n, 2 * A if K.continuous else A)
        dev = values.device
        tok = torch.empty(b, n, L.LOSS_TOK, device=dev, dtype=torch.float32)
        stats = torch.zeros(L.LOSS_STATS, device=dev, dtype=torch.float32)
        d = L.LossDesc(b=b, n=n, A=A, B=B, S1=S1, continuous=int(K.continuous), squash=int(K.squash),
                       hl_reduction_mean=int(K.hl_mean), eps_clip=K.eps_clip, value_clip=K.value_clip,
                       entropy_weight=K.entropy_weight, w_actor=K.w_actor, w_critic=K.w_critic,
                       w_autoreg=K.w_autoreg, lo=K.lo, hi=K.hi, sigma=K.sigma)
        keep = [raw_actions, values, pred_raw, done_logit, tok, stats]
        fields = dict(raw_actions=raw_actions, values=values, pred_raw=pred_raw, done_logit=done_logit,
                      actions=None if K.continuous else K.actions, actions_f=K.actions if K.continuous else None,
                      old_logp=K.old_logp, returns=K.returns, old_values=K.old_values, dones=K.dones, lens=K.lens,
                      real=K.real, support=K.support, centers=K.centers, tok=tok, stats=stats)
        for name, t in fields.items():
            if t is not None:
                assert t.is_cuda and t.is_contiguous(), name
                setattr(d, name, t.data_ptr())
        L.check(lib.xtrl_loss_fwd(C.byref(d), L.stream()), 'loss_fwd')
        ctx.desc = d
        ctx.keep = keep + [K]
        ctx.shapes = (raw_actions.shape, values.shape, pred_raw.shape, done_logit.shape)
        ctx.mark_non_differentiable(stats)
        return stats[L.LS['loss']].clone(), stats

    @staticmethod
    def backward(ctx, gloss, gstats):
        lib = L.lib()
        d = ctx.desc
        sa, sv, sp, sd = ctx.shapes
        dev = gloss.device
        g_raw = torch.empty(sa, device=dev, dtype=torch.float32)
        g_val = torch.empty(sv, device=dev, dtype=torch.float32)
        g_pred = torch.empty(sp, device=dev, dtype=torch.float32)
        g_done = torch.empty(sd, device=dev, dtype=torch.float32)
        d.d_raw_actions, d.d_values, d.d_pred_raw, d.d_done_logit = (t.data_ptr() for t in (g_raw, g_val, g_pred, g_done))
        # the upstream gradient is 1 for loss.backward(); a different scalar is folded in afterwards
        L.check(lib.xtrl_loss_bwd(C.byref(d), 1.0, L.stream()), 'loss_bwd')
        if not (isinstance(gloss, torch.Tensor) and gloss.numel() == 1):
            raise RuntimeError('fused loss expects a scalar upstream gradient')
        s = gloss.reshape(())
        return g_raw * s, g_val * s, g_pred * s, g_done * s, None


def fused_loss(raw_actions, values, pred_raw, done_logit, consts: LossConsts):
    return LossFn.apply(raw_actions, values, pred_raw, done_logit, consts)


# --------------------------------------------------------------------------------------------
# HL-Gauss + GAE, optimiser
# --------------------------------------------------------------------------------------------


def hlgauss_gae(logits, rewards, bounds, centers, n, gamma, lam, boot=None, lens=None):
    """logits [E, T, B] (uses [:, :n]), rewards / bounds [E, T] -> (values, returns) [E, n].
    ``boot`` [E] (NaN = none) with ``lens`` [E] int32: truncation-bootstrap values at index lens."""
    lib = L.lib()
    E, T, B = logits.shape
    assert rewards.shape == (E, T) and bounds.shape == (E, T) and bounds.dtype == torch.uint8 and n <= T
    if boot is not None:
        assert boot.shape == (E,) and boot.dtype == torch.float32 and boot.is_contiguous()
        assert lens is not None and lens.shape == (E,) and lens.dtype == torch.int32 and lens.is_contiguous()
    values = torch.empty(E, n, device=logits.device, dtype=torch.float32)
    returns = torch.empty_like(values)
    gl = float(torch.tensor(gamma * lam, dtype=torch.float32))
    L.check(lib.xtrl_hlgauss_gae(L.ptr(logits), T * B, L.ptr(rewards), L.ptr(bounds), T, L.ptr(centers),
                                 L.ptr(values), L.ptr(returns), E, n, B, float(gamma), gl, L.ptr(boot),
                                 L.ptr(lens if boot is not None else None), L.stream()), 'hlgauss_gae')
    return values, returns


def grad_norm(flat_grad, max_norm, ws, out):
    L.check(L.lib().xtrl_grad_norm(L.ptr(flat_grad), flat_grad.numel(), L.ptr(ws), float(max_norm), L.ptr(out),
                                   L.stream()), 'grad_norm')


def adopt_chunks(seg, chunk=2048):
    """[n_chunks][3] (start, end, tensor) pieces of the flat buffer, one workgroup each."""
    offs = seg.tolist()
    rows = []
    for s_, (a, b) in enumerate(zip(offs[:-1], offs[1:])):
        for st in range(a, b, chunk):
            rows.append((st, min(st + chunk, b), s_))
    return torch.tensor(rows, dtype=torch.int64, device=seg.device)


def adopt_atan2(p, g, m, v, p_init, seg, chunks, seg_ws, clip, *, lr, init_lr, betas, a, b, weight_decay, regen_rate,
                cautious, first_step):
    L.check(L.lib().xtrl_adopt_atan2(L.ptr(p), L.ptr(g), L.ptr(m), L.ptr(v), L.ptr(p_init), p.numel(), L.ptr(chunks),
                                     chunks.shape[0], L.ptr(seg), seg.numel() - 1, L.ptr(seg_ws), L.ptr(clip), lr,
                                     init_lr, betas[0], betas[1], a, b, weight_decay, regen_rate, cautious,
                                     int(first_step), L.stream()), 'adopt_atan2')


def ema_lerp(ema, p, weight):
    L.check(L.lib().xtrl_ema_lerp(L.ptr(ema), L.ptr(p), p.numel(), float(weight), L.stream()), 'ema_lerp')
