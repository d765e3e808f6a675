"""Hand-scheduled learn step: one minibatch forward + loss + backward through libxtrl_hip without
autograd (xtrl_train_forward / xtrl_loss_fwd / xtrl_loss_bwd / xtrl_train_backward).

Replaces, for Agent.learn (x_transformers_rl.py:880-1023), the per-minibatch
``model(...)`` -> losses -> ``loss.backward()`` sequence.  Activations live in buffers allocated
once for the largest minibatch (``b_max`` episodes x ``n_max`` steps, token-major) and reused by
every minibatch; gradients are accumulated into the flat gradient buffer of ``FlatParams``.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib as L
from .params import FlatParams


def ld_ff(ff):
    """Row stride of the [T][ff] feed-forward activations (XtrlTrainDesc.ld_ff): ff + 16 when the row
    is a multiple of 1 KiB (a power-of-two stride puts the FF1 epilogue's two store streams on the same
    memory channels: 93 -> 82 us a launch at C3's ff = 1024, tools/epi_gemm_lab.cpp)."""
    return ff + 16 if ff % 256 == 0 else ff


def _off(flat, name):
    return flat.index[name][0] if name in flat.index else -1


def _span_off(flat, names):
    flat.span(names)   # asserts adjacency
    return flat.index[names[0]][0]


def _compact_bufs(D, c, T, dev, b_max, n_max):
    """The world-model heads' valid-row buffers (XtrlTrainDesc.Tv): row list / inverse and the compact
    operands, T rows each (the most a minibatch can have valid)."""
    d, ldp, S1x2 = c.dim, c.dim + 4, 2 * (c.state_dim + 1)
    f32 = dict(device=dev, dtype=torch.float32)
    bufs = dict(vrows=torch.empty(T, device=dev, dtype=torch.int32), vinv=torch.empty(T, device=dev, dtype=torch.int32),
                ewa_v=torch.empty(T, 2 * d, **f32), hp_v=torch.empty(T, ldp, **f32), zp_v=torch.empty(T, ldp, **f32),
                pred_v=torch.empty(T, S1x2, **f32), d_pred_v=torch.empty(T, S1x2, **f32),
                dzp_v=torch.empty(T, ldp, **f32), dewa_v=torch.empty(T, 2 * d, **f32))
    for k, t in bufs.items():
        setattr(D, k, t.data_ptr())
    D.Tv = 0
    # the packed learn step's episode row offsets and its packed inputs / outputs (allocated on first use)
    bufs['ep_off'] = torch.zeros(b_max + 1, device=dev, dtype=torch.int32)
    D.ep_off, D.packed, D.pack_ws, D.pack_ws_floats = bufs['ep_off'].data_ptr(), 0, None, 0
    # long episodes (n > 128, dh 16): the attention backward's per-key-tile dQ partials (xtrl_attn_bwd_part)
    D.dq_part, D.dq_part_floats = None, 0
    if n_max > 128 and c.dim_head == 16:
        nf = int(L.lib().xtrl_attn_bwd_part_floats(b_max, c.heads, n_max, c.dim_head))
        bufs['dq_part'] = torch.empty(nf, **f32)
        D.dq_part, D.dq_part_floats = bufs['dq_part'].data_ptr(), nf
    return bufs


def _heads_desc(D, c, flat):
    """Offsets of the heads every policy body shares (xtrl.py:533-557, fractal_rl.py:586-619)."""
    off = lambda n: _off(flat, n)
    if c.continuous:
        D.act_emb, D.act_emb_b = off('action_embeds.weight'), off('action_embeds.bias')
    else:
        D.act_emb, D.act_emb_b = off('action_embeds.embed.weight'), -1
    D.reward_embed, D.w_se, D.b_se = off('reward_embed'), off('to_state_embed.weight'), off('to_state_embed.bias')
    D.w_pd = _span_off(flat, ['to_pred.0.weight', 'to_pred_done.0.weight'])
    D.b_pd = _span_off(flat, ['to_pred.0.bias', 'to_pred_done.0.bias'])
    D.w_pred2, D.b_pred2 = off('to_pred.2.weight'), off('to_pred.2.bias')
    D.w_lat, D.b_lat = off('latent_to_embed.weight'), off('latent_to_embed.bias')
    D.w_h1 = _span_off(flat, ['action_head.0.weight', 'critic_head.0.weight'])
    D.b_h1 = _span_off(flat, ['action_head.0.bias', 'critic_head.0.bias'])
    D.w_a2, D.b_a2 = off('action_head.2.weight'), off('action_head.2.bias')
    D.w_c2, D.b_c2 = off('critic_head.2.weight'), off('critic_head.2.bias')


class FusedTrainStep:
    def __init__(self, model, flat: FlatParams, ws: torch.Tensor, b_max: int, n_max: int):
        c = model.cfg
        self.model, self.flat, self.cfg, self.ws = model, flat, c, ws
        dev = flat.flat.device
        self.dev = dev
        d, H, dh, L_ = c.dim, c.heads, c.dim_head, c.depth
        I, ff, B = H * dh, c.dim * c.ff_mult, c.num_bins
        S, A = c.state_dim, c.num_actions
        n_out = A * (2 if c.continuous else 1)
        T = b_max * n_max
        self.b_max, self.n_max, self.T_max = b_max, n_max, T
        self.inv_freq = model.transformer.attn_layers.rotary_pos_emb.inv_freq.to(dev).contiguous()
        rot = 2 * self.inv_freq.numel()
        f32 = dict(device=dev, dtype=torch.float32)
        E = lambda *shape: torch.empty(*shape, **f32)
        off = lambda name: flat.index[name][0] if name in flat.index else -1
        pre = 'transformer.attn_layers.layers.'

        def span_off(names):
            a0 = flat.index[names[0]][0]
            flat.span(names)   # asserts adjacency
            return a0

        self.layers_py = []
        self.ld_ff = lff = ld_ff(ff)
        glu = bool(getattr(c, 'ff_glu', False))
        # ff_glu: u holds the GLU projection's output [T][2 ff] (stride lu2), dff its gradient planes
        lu2 = ld_ff(2 * ff) if glu else lff
        layers = (L.TrainLayer * L_)()
        X = [E(T, d) for _ in range(L_ + 1)]
        max_qkv = 0
        nw = 'g' if c.rms_norm else 'gamma'   # x-transformers RMSNorm.g / LayerNorm.gamma
        for li in range(L_):
            mix = bool(c.value_residual and c.learned_mix and li > 0)
            pa, pf = f'{pre}{2 * li}.', f'{pre}{2 * li + 1}.'
            wn = [pa + '1.to_q.weight', pa + '1.to_k.weight', pa + '1.to_v.weight']
            wn += [pa + '1.to_v_gate.weight'] if c.gate_values else []
            wn += [pa + '1.to_value_residual_mix.0.weight'] if mix else []
            bn = ([pa + '1.to_v_gate.bias'] if c.gate_values else []) + \
                 ([pa + '1.to_value_residual_mix.0.bias'] if mix else [])
            n_qkv = 3 * I + (I if c.gate_values else 0) + (H if mix else 0)
            max_qkv = max(max_qkv, n_qkv)
            bufs = dict(x_attn=X[li], x_ff=E(T, d), xn_attn=E(T, d), xn_ff=E(T, d), st_attn=E(T, 2), st_ff=E(T, 2),
                        proj=E(T, n_qkv), qkv=E(T, 3 * I), o=E(T, I), lse=E(b_max * H * n_max), u=E(T, lu2),
                        hd=E(T, lff))
            bufs['og'] = E(T, I) if c.gate_values else bufs['o']
            self.layers_py.append(bufs)
            Ly = layers[li]
            Ly.ln_attn, Ly.w_proj = off(pa + '0.0.' + nw), span_off(wn)
            Ly.b_proj = span_off(bn) if bn else -1
            Ly.w_out, Ly.ln_ff = off(pa + '1.to_out.weight'), off(pf + '0.0.' + nw)
            f1 = pf + ('1.ff.0.proj.' if glu else '1.ff.0.0.')
            Ly.w_ff1, Ly.b_ff1 = off(f1 + 'weight'), off(f1 + 'bias')
            Ly.w_ff2, Ly.b_ff2 = off(pf + '1.ff.2.weight'), off(pf + '1.ff.2.bias')
            Ly.n_qkv, Ly.mix = n_qkv, int(mix)
            for k, t in bufs.items():
                setattr(Ly, k, t.data_ptr())
        self.layers = layers
        self.X = X
        ldp = d + 4
        self.buf = dict(x_final=X[L_], st_final=E(T, 2), ac_in=E(T, c.in_dim), ewa=E(T, 2 * d), zp=E(T, ldp),
                        hp=E(T, ldp), z1=E(T, 4 * d), h1=E(T, 4 * d), lat_e=E(max(b_max, 1), d),
                        raw=E(T, n_out), values=E(T, B), pred=E(T, 2 * (S + 1)), done=E(T),
                        d_raw=E(T, n_out), d_values=E(T, B), d_pred=E(T, 2 * (S + 1)), d_done=E(T),
                        dx=E(L_ + 1, T, d), dx2=E(L_, T, d), dxn=E(T, d), dff=E(L_, T, lu2), dproj=E(L_, T, max_qkv),
                        dog=E(T, I), dvfirst=E(T, I),
                        dz1=E(T, 4 * d), dac=E(T, c.in_dim), dzp=E(T, ldp), dewa=E(T, 2 * d),
                        delta=E(b_max * H * n_max))
        # the library states its own partial-sum needs (LayerNorm-backward row blocks, column sums)
        if glu:
            self.buf['glu_dh'] = E(T, lff)
        part = max(256 * max((2 if glu else 1) * ff, 4 * d, B, max_qkv), 1024 * max(A, 1) * d,
                   int(L.lib().xtrl_train_part_floats(T, b_max, d, A)))
        self.buf['part'] = E(part)
        self.tok = torch.empty(b_max, n_max, L.LOSS_TOK, **f32)
        self.stats = torch.zeros(L.LOSS_STATS, **f32)

        D = L.TrainDesc()
        D.S, D.A, D.d, D.L, D.H, D.dh, D.ff, D.B = S, A, d, L_, H, dh, ff, B
        D.in_dim, D.n_out, D.G = c.in_dim, n_out, c.dim_gene if c.evolutionary else 0
        D.continuous, D.evolutionary, D.gate_values, D.rot_dim = int(c.continuous), int(c.evolutionary), \
            int(c.gate_values), rot
        D.frac_head_grad = float(c.frac_head_grad)
        D.attn_scale = float(c.qk_norm_scale) if c.qk_norm else float(dh ** -0.5)
        D.qk_norm, D.xpos_base = int(c.qk_norm), float(c.xpos_scale_base) if c.rotary_xpos else 0.
        D.flat, D.grad = flat.flat.data_ptr(), flat.grad.data_ptr()
        D.w_pin = off('transformer.project_in.weight')
        _heads_desc(D, c, flat)
        D.ln_final = off('transformer.attn_layers.final_norm.' + nw)
        D.rms_norm = int(c.rms_norm)
        D.inv_freq = self.inv_freq.data_ptr()
        for k, t in self.buf.items():
            setattr(D, k, t.data_ptr())
        D.part_floats = self.buf['part'].numel()
        D.ws, D.ws_floats = ws.data_ptr(), ws.numel()
        D.layers = C.cast(layers, C.POINTER(L.TrainLayer))
        D.ld_ff = lff
        D.scratch_per_layer = 1   # per-layer backward planes (no mid-backward stream waits)
        D.ff_glu, D.ld_u2 = int(glu), (lu2 if glu else 0)
        self.cbuf = _compact_bufs(D, c, T, dev, b_max, n_max)
        self.D = D

    # ------------------------------------------------------------------------------------------
    def forward(self, swr, prev_action, next_action, latent, lens, reward_keep, seed, attn_offset, ff_offset,
                dropout, Tv=0, packed=False):
        """swr [b][n][S+1] normalised states | previous reward; actions [b][n] int32 (discrete) or
        [b][n][A] float (continuous); latent [b][G] or None; lens [b] int32.  ``Tv``: the number of
        valid tokens (sum of min(lens, n), known on the host) — the world-model heads then run on
        those rows only and pred / done hold zeros on the padding; 0: every row.  ``packed``: the
        whole step on the Tv valid tokens (XtrlTrainDesc.packed; per-token critic reduction only —
        Agent(packed_learn=True)); the outputs come back in the [b][n] layout, zeros on the padding.
        Returns views raw [b][n][n_out], values [b][n][B], pred [b][n][2(S+1)], done [b][n]."""
        self._bind_inputs(swr, prev_action, next_action, latent, lens, reward_keep, seed, attn_offset, ff_offset,
                          dropout, Tv)
        D = self.D
        D.packed = 0
        if packed:
            assert 0 < Tv <= D.b * D.n, (Tv, D.b, D.n)
            D.Tv, D.packed = int(Tv), 1
            if self.cbuf.get('pack_ws') is None:
                c = self.cfg
                nf = int(L.lib().xtrl_train_pack_floats(self.T_max, c.state_dim, c.num_actions, D.n_out, c.num_bins))
                self.cbuf['pack_ws'] = torch.empty(nf, device=self.dev, dtype=torch.float32)
                D.pack_ws, D.pack_ws_floats = self.cbuf['pack_ws'].data_ptr(), nf
        L.check(L.lib().xtrl_train_forward(C.byref(self.D), L.stream()), 'train_forward')
        return self._outputs()

    def _bind_inputs(self, swr, prev_action, next_action, latent, lens, reward_keep, seed, attn_offset, ff_offset,
                     dropout, Tv=0):
        c, D = self.cfg, self.D
        b, n = swr.shape[0], swr.shape[1]
        assert b <= self.b_max and n <= self.n_max, (b, n, self.b_max, self.n_max)
        assert 0 <= Tv <= b * n, (Tv, b, n)
        D.Tv = int(Tv) if Tv < b * n else 0
        for t in (swr, prev_action, next_action, lens):
            assert t.is_cuda and t.is_contiguous()
        self._keep = [swr, prev_action, next_action, latent, lens]
        D.b, D.n = b, n
        D.dropout, D.reward_keep = float(dropout), float(reward_keep)
        D.seed, D.attn_offset, D.ff_offset = int(seed) & (2 ** 64 - 1), int(attn_offset) & 0xFFFFFFFF, \
            int(ff_offset) & 0xFFFFFFFF
        D.swr, D.lens = swr.data_ptr(), lens.data_ptr()
        if c.continuous:
            D.prev_action_f, D.next_action_f, D.prev_action, D.next_action = prev_action.data_ptr(), \
                next_action.data_ptr(), None, None
        else:
            assert prev_action.dtype == torch.int32 and next_action.dtype == torch.int32
            D.prev_action, D.next_action, D.prev_action_f, D.next_action_f = prev_action.data_ptr(), \
                next_action.data_ptr(), None, None
        D.latent = latent.contiguous().data_ptr() if latent is not None else None
        if latent is not None:
            self._keep.append(latent.contiguous())
            D.latent = self._keep[-1].data_ptr()

    def _outputs(self):
        b, n = self.D.b, self.D.n
        T = b * n
        bf = self.buf
        return (bf['raw'][:T].view(b, n, -1), bf['values'][:T].view(b, n, -1), bf['pred'][:T].view(b, n, -1),
                bf['done'][:T].view(b, n))

    def loss(self, K, stats=None):
        """Fused loss forward + backward (upstream gradient 1) into the d_* buffers.
        Returns the stats tensor (XTRL_LS_* slots)."""
        c, D = self.cfg, self.D
        b, n = D.b, D.n
        T = b * n
        bf = self.buf
        S1 = c.state_dim + 1
        A = c.num_actions
        # ``stats``: a caller-owned row (every XTRL_LS_* slot is written by the loss kernels), else
        # the step's own buffer, cloned on return since the next minibatch reuses it
        own = stats is None
        if own:
            self.stats.zero_()
            stats = self.stats
        d = L.LossDesc(b=b, n=n, A=A, B=c.num_bins, S1=S1, continuous=int(K.continuous), squash=int(K.squash),
                       hl_reduction_mean=int(K.hl_mean), eps_clip=K.eps_clip, value_clip=K.value_clip,
                       entropy_weight=K.entropy_weight, w_actor=K.w_actor, w_critic=K.w_critic,
                       w_autoreg=K.w_autoreg, lo=K.lo, hi=K.hi, sigma=K.sigma)
        fields = dict(raw_actions=bf['raw'], values=bf['values'], pred_raw=bf['pred'], done_logit=bf['done'],
                      actions=None if K.continuous else K.actions, actions_f=K.actions if K.continuous else None,
                      old_logp=K.old_logp, returns=K.returns, old_values=K.old_values, dones=K.dones, lens=K.lens,
                      real=K.real, support=K.support, centers=K.centers, tok=self.tok, stats=stats,
                      d_raw_actions=bf['d_raw'], d_values=bf['d_values'], d_pred_raw=bf['d_pred'],
                      d_done_logit=bf['d_done'])
        for name, t in fields.items():
            if t is not None:
                assert t.is_cuda and t.is_contiguous(), name
                setattr(d, name, t.data_ptr())
        lib = L.lib()
        L.check(lib.xtrl_loss_fwd(C.byref(d), L.stream()), 'loss_fwd')
        L.check(lib.xtrl_loss_bwd(C.byref(d), 1.0, L.stream()), 'loss_bwd')
        del T
        return stats.clone() if own else stats

    def backward(self, grad_events=None):
        """``grad_events``: ctypes array of 2 (L + 2) HIP event handles recorded per gradient bucket
        (distributed.BucketAllReduce), or None."""
        self.D.grad_events = C.cast(grad_events, C.POINTER(C.c_void_p)) if grad_events is not None else None
        L.check(L.lib().xtrl_train_backward(C.byref(self.D), L.stream()), 'train_backward')


class FractalTrainStep(FusedTrainStep):
    """The hand-scheduled learn step of the causal fractal policy body (fractal.FractalPolicyActorCritic,
    xtrl_fractal_train_forward / _backward): the same minibatch interface, loss and heads as the
    decoder's FusedTrainStep; the encoder per level: q|k|v GEMM, causal flash attention, three
    post-norm residual blocks with nn.LayerNorm formed in the GEMM epilogues, the causal running
    mean, level projection and global-state update, then the final aggregation."""

    def __init__(self, model, flat: FlatParams, ws: torch.Tensor, b_max: int, n_max: int):
        c = model.cfg
        self.model, self.flat, self.cfg, self.ws = model, flat, c, ws
        dev = flat.flat.device
        self.dev = dev
        d, H, dh, Lv = c.dim, c.heads, c.dim_head, model.levels
        I, ff, B = H * dh, c.dim * c.ff_mult, c.num_bins
        S, A = c.state_dim, c.num_actions
        n_out = A * (2 if c.continuous else 1)
        T = b_max * n_max
        self.b_max, self.n_max, self.T_max = b_max, n_max, T
        f32 = dict(device=dev, dtype=torch.float32)
        E = lambda *shape: torch.empty(*shape, **f32)
        off = lambda name: _off(flat, name)
        enc = 'fractal_encoder.'
        le0 = off(enc + 'level_embedding.level_embeds')
        levels = (L.FractalTrainLevel * Lv)()
        self.levels_py = []
        self.ld_ff = lff = ld_ff(ff)
        for li in range(Lv):
            pre = model.block_prefix(li)
            V = levels[li]
            V.w_qkv = _span_off(flat, [pre + 'self_attn.to_q.weight', pre + 'self_attn.to_k.weight',
                                       pre + 'self_attn.to_v.weight'])
            V.w_out, V.w_gv, V.w_go = off(pre + 'self_attn.to_out.weight'), off(pre + 'global_attn.to_v.weight'), \
                off(pre + 'global_attn.to_out.weight')
            for k in (1, 2, 3):
                setattr(V, f'ln{k}_w', off(pre + f'norm{k}.weight'))
                setattr(V, f'ln{k}_b', off(pre + f'norm{k}.bias'))
            V.w_ff1, V.b_ff1 = off(pre + 'ff.ff.0.0.weight'), off(pre + 'ff.ff.0.0.bias')
            V.w_ff2, V.b_ff2 = off(pre + 'ff.ff.2.weight'), off(pre + 'ff.ff.2.bias')
            V.w_proj, V.b_proj = off(enc + f'level_projections.{li}.weight'), off(enc + f'level_projections.{li}.bias')
            V.level_embed = le0 + li * d
            bufs = dict(xin=E(T, d), qkv=E(T, 3 * I), o=E(T, I), lse=E(b_max * H * n_max), s1=E(T, d), x1=E(T, d),
                        st1=E(T, 2), g=E(T, d), gv=E(T, I), s2=E(T, d), x2=E(T, d), st2=E(T, 2), h=E(T, lff),
                        u=E(T, lff), s3=E(T, d), x3=E(T, d), st3=E(T, 2), mean=E(T, d))
            for k, t in bufs.items():
                setattr(V, k, t.data_ptr())
            self.levels_py.append(bufs)
        self.levels = levels
        ldp = d + 4
        self.buf = dict(ac_in=E(T, c.in_dim), ewa=E(T, 2 * d), zp=E(T, ldp), hp=E(T, ldp), z1=E(T, 4 * d),
                        h1=E(T, 4 * d), lat_e=E(max(b_max, 1), d), raw=E(T, n_out), values=E(T, B),
                        pred=E(T, 2 * (S + 1)), done=E(T), d_raw=E(T, n_out), d_values=E(T, B),
                        d_pred=E(T, 2 * (S + 1)), d_done=E(T), dz1=E(T, 4 * d), dac=E(T, c.in_dim), dzp=E(T, ldp),
                        dewa=E(T, 2 * d), delta=E(b_max * H * n_max))
        # LayerNorm backward: d gamma and d beta partial rows side by side
        part = max(256 * max(ff, 4 * d, B, 3 * I), 1024 * max(A, 1) * d,
                   2 * int(L.lib().xtrl_train_part_floats(T, b_max, d, A)))
        self.buf['part'] = E(part)
        self.tok = torch.empty(b_max, n_max, L.LOSS_TOK, **f32)
        self.stats = torch.zeros(L.LOSS_STATS, **f32)
        self.scale_embeds = model.fractal_encoder.level_embedding.scale_embeds[:Lv].to(dev).float().contiguous()
        self.fbuf = dict(scale_embeds=self.scale_embeds, le=E(Lv, d), bias0=E(d), cat=E(T, (Lv + 1) * d),
                         hfa=E(T, 2 * d), dxa=E(T, d), dxb=E(T, d), ds=E(3 * Lv + 1, T, d), dmean=E(T, d),
                         dga=E(Lv, T, d), dgv=E(Lv, T, I), dz=E(Lv, T, lff), dqkv=E(Lv, T, 3 * I), dob=E(T, I),
                         dcat=E(T, (Lv + 1) * d), dhfa=E(T, 2 * d))

        D = L.TrainDesc()
        D.S, D.A, D.d, D.L, D.H, D.dh, D.ff, D.B = S, A, d, Lv, H, dh, ff, B
        D.in_dim, D.n_out, D.G = c.in_dim, n_out, c.dim_gene if c.evolutionary else 0
        D.continuous, D.evolutionary, D.gate_values, D.rot_dim = int(c.continuous), int(c.evolutionary), 0, 0
        D.frac_head_grad, D.attn_scale = float(c.frac_head_grad), float(dh ** -0.5)
        D.flat, D.grad = flat.flat.data_ptr(), flat.grad.data_ptr()
        D.w_pin = off(enc + 'input_embed.weight')
        _heads_desc(D, c, flat)
        D.ln_final = -1
        for k, t in self.buf.items():
            setattr(D, k, t.data_ptr())
        D.part_floats = self.buf['part'].numel()
        D.ws, D.ws_floats = ws.data_ptr(), ws.numel()
        D.layers = None
        D.ld_ff = lff
        self.cbuf = _compact_bufs(D, c, T, dev, b_max, n_max)
        self.D = D
        Fd = L.FractalTrainDesc()
        Fd.levels = Lv
        Fd.b_in = off(enc + 'input_embed.bias')
        Fd.g_init = off(enc + 'global_state_init')
        Fd.w_gu, Fd.b_gu = off(enc + 'global_state_update.weight'), off(enc + 'global_state_update.bias')
        Fd.w_fa0, Fd.b_fa0 = off(enc + 'final_aggregation.0.weight'), off(enc + 'final_aggregation.0.bias')
        Fd.w_fa2, Fd.b_fa2 = off(enc + 'final_aggregation.2.weight'), off(enc + 'final_aggregation.2.bias')
        for k, t in self.fbuf.items():
            setattr(Fd, k, t.data_ptr())
        Fd.level = C.cast(levels, C.POINTER(L.FractalTrainLevel))
        self.Fd = Fd

    def forward(self, swr, prev_action, next_action, latent, lens, reward_keep, seed, attn_offset, ff_offset,
                dropout, Tv=0, packed=False):
        assert not packed, 'the packed learn step is built for the decoder policy body'
        self._bind_inputs(swr, prev_action, next_action, latent, lens, reward_keep, seed, attn_offset, ff_offset,
                          dropout, Tv)
        L.check(L.lib().xtrl_fractal_train_forward(C.byref(self.D), C.byref(self.Fd), L.stream()),
                'fractal_train_forward')
        return self._outputs()

    def backward(self, grad_events=None):
        """``grad_events``: ctypes array of 2 (levels + 2) HIP event handles recorded per gradient
        bucket (FractalPolicyActorCritic.flat_buckets_names), or None."""
        self.D.grad_events = C.cast(grad_events, C.POINTER(C.c_void_p)) if grad_events is not None else None
        L.check(L.lib().xtrl_fractal_train_backward(C.byref(self.D), C.byref(self.Fd), L.stream()),
                'fractal_train_backward')


def ff_dropout_mask(M, N, p, seed, offset, device, layer=0):
    """The feed-forward dropout keep mask the fused step uses (uint8 [M][N]) — reference mode."""
    m = torch.empty(M, N, device=device, dtype=torch.uint8)
    L.check(L.lib().xtrl_ff_dropout_mask(L.ptr(m), M, N, float(p), int(seed) & (2 ** 64 - 1),
                                         int(offset) & 0xFFFFFFFF, int(layer), L.stream()), 'ff_dropout_mask')
    return m


class BatchGather:
    """Device minibatch assembly (xtrl_minibatch_gather) into persistent [b_max][n_max] buffers."""

    def __init__(self, cfg, b_max, n_max, device, rs_m=None):
        """``rs_m``: optional [S+1] output buffer of the minibatch RSNorm mean (the tail of the
        learner's extended gradient buffer, so the DP all-reduce carries it)."""
        c = cfg
        self.c, self.b_max, self.n_max = c, b_max, n_max
        S, A, B = c.state_dim, c.num_actions, c.num_bins
        f32, i32, u8 = dict(device=device, dtype=torch.float32), dict(device=device, dtype=torch.int32), \
            dict(device=device, dtype=torch.uint8)
        T = b_max * n_max
        self.buf = dict(swr=torch.empty(T * (S + 1), **f32), old_logp=torch.empty(T * (A if c.continuous else 1), **f32),
                        mb_returns=torch.empty(T, **f32), old_values=torch.empty(T * B, **f32),
                        dones=torch.empty(T, **u8), mb_lens=torch.empty(b_max, **i32),
                        rs_part=torch.empty(64 * (S + 2), **f32),
                        rs_m=rs_m if rs_m is not None else torch.empty(S + 1, **f32))
        assert self.buf['rs_m'].numel() == S + 1 and self.buf['rs_m'].is_contiguous()
        if c.continuous:
            self.buf.update(prev_action_f=torch.empty(T * A, **f32), action_f=torch.empty(T * A, **f32))
        else:
            self.buf.update(prev_action=torch.empty(T, **i32), action=torch.empty(T, **i32))

    def __call__(self, traj, returns, lens, idx, rs_mean, rs_var, n):
        c, bf = self.c, self.buf
        b = idx.shape[0]
        assert b <= self.b_max and n <= self.n_max
        N, Tmax = traj['rewards'].shape
        S, A, B = c.state_dim, c.num_actions, c.num_bins
        D = L.BatchDesc(N=N, Tmax=Tmax, n=n, b=b, S=S, A=A, B=B, continuous=int(c.continuous))
        src = dict(states=traj['states'], actions=None if c.continuous else traj['actions'],
                   actions_f=traj['actions_f'] if c.continuous else None, rewards=traj['rewards'], logp=traj['logp'],
                   bounds=traj['bounds'], values=traj['values'], returns=returns, lens=lens, idx=idx,
                   rs_mean=rs_mean, rs_var=rs_var)
        for k, t in src.items():
            if t is not None:
                assert t.is_cuda and t.is_contiguous(), k
                setattr(D, k, t.data_ptr())
        for k, t in bf.items():
            setattr(D, k, t.data_ptr())
        L.check(L.lib().xtrl_minibatch_gather(C.byref(D), L.stream()), 'minibatch_gather')
        T = b * n
        out = dict(swr=bf['swr'][:T * (S + 1)].view(b, n, S + 1), returns=bf['mb_returns'][:T].view(b, n),
                   old_values=bf['old_values'][:T * B].view(b, n, B), dones=bf['dones'][:T].view(b, n),
                   lens=bf['mb_lens'][:b], rs_m=bf['rs_m'])
        if c.continuous:
            out.update(prev_action=bf['prev_action_f'][:T * A].view(b, n, A), action=bf['action_f'][:T * A].view(b, n, A),
                       old_logp=bf['old_logp'][:T * A].view(b, n, A))
        else:
            out.update(prev_action=bf['prev_action'][:T].view(b, n), action=bf['action'][:T].view(b, n),
                       old_logp=bf['old_logp'][:T].view(b, n))
        return out


def rsnorm_update(mean, var, m, t):
    L.check(L.lib().xtrl_rsnorm_update(L.ptr(mean), L.ptr(var), L.ptr(m), mean.numel(), int(t), L.stream()),
            'rsnorm_update')
