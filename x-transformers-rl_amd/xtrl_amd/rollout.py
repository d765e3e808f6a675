"""Device-resident vectorised rollout (replaces Learner.forward's batch-1 loop, xtrl.py:1204-1356).

One ``RolloutEngine`` owns, for a fixed (E envs x Tmax steps) shape:
  * packed decode weights (refreshed from the EMA model once per learning update — the rollout
    policy is constant for the whole update, xtrl.py:1194),
  * per-layer KV caches [E][H][Tmax][dh], env state, trajectory buffers [E][Tmax][.],
  * the ctypes ``XtrlDecodeDesc`` pointing at all of them.
``run()`` drives ``xtrl_decode_step`` for t = 0..Tmax-1, either eagerly or by replaying a captured
hipGraph of the whole rollout (the graph is reusable across updates because every buffer is
persistent and the seed / update index live in device memory).

Per step only the live episodes are decoded: the step's embedding kernel compacts them into
rows 0..n-1 (``live_rows`` / ``live_count``, double-buffered by step parity) and every later
kernel of the step reads the live count from device memory, so the captured graph needs no host
sync and terminated episodes cost nothing.
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import os
import time

import numpy as np
import torch
import torch.nn.functional as F

from . import _lib as L
from . import ops
from .model import WorldModelActorCritic, norm_gain

SIM_README, SIM_LANDER, SIM_HOST = 0, 1, -1


def _r4(n):
    return (n + 3) & ~3


class RolloutEngine:
    def __init__(self, model: WorldModelActorCritic, E: int, Tmax: int, *, sim_mode=SIM_LANDER, hazard_log2=6,
                 clamp=None, use_graph=False, cfg=None):
        c = cfg if cfg is not None else model.cfg
        dev = next(model.parameters()).device
        self.c, self.E, self.T, self.dev = c, E, Tmax, dev
        self.sim_mode, self.use_graph = sim_mode, use_graph
        d, H, dh, S, A, B = c.dim, c.heads, c.dim_head, c.state_dim, c.num_actions, c.num_bins
        I = H * dh
        self.n_qkv = 3 * I + (I if c.gate_values else 0) + (H if (c.value_residual and c.learned_mix) else 0)
        ff = d * c.ff_mult
        nA = 2 * A if c.continuous else A
        f32, i32, u8 = torch.float32, torch.int32, torch.uint8
        z = lambda *s, dt=f32: torch.zeros(*s, device=dev, dtype=dt)
        # env / episode state
        self.state, self.prev_action, self.prev_action_f = z(E, S), z(E, dt=i32), z(E, A)
        self.prev_reward, self.alive, self.lens = z(E), z(E, dt=u8), z(E, dt=i32)
        self.cum_reward = z(E, dt=torch.float64)
        self.episode_of_slot = z(E, dt=i32)
        self.slot_of_row = z(E, dt=i32)   # global pair index per row (non-contiguous shards)
        self.rng = z(2, dt=torch.int64)
        self.live_rows, self.live_count = z(2, E, dt=i32), z(2, dt=i32)
        self.lat_embed = z(E, d) if c.evolutionary else None
        # trajectory
        self.traj = dict(states=z(E, Tmax, S), actions=z(E, Tmax, dt=i32), actions_f=z(E, Tmax, A) if c.continuous else None,
                         logp=z(E, Tmax, A) if c.continuous else z(E, Tmax), rewards=z(E, Tmax),
                         bounds=z(E, Tmax, dt=u8), values=z(E, Tmax, B))
        # scratch
        self.x, self.qkv, self.att = z(E, d), z(E, self.n_qkv), z(E, I)
        glu = bool(getattr(c, 'ff_glu', False))   # world_model['ff_glu']: FF1 is the GLU projection [2 ff][d]
        self.hff, self.ac_in, self.logits, self.v1 = z(E, max(2 * ff if glu else ff, 4 * d)), z(E, c.in_dim), \
            z(E, nA), z(E, I)
        self.hglu = z(E, ff) if glu else None
        self.xn = z(E, d)
        # one-launch feed-forward (k_mlp): per 16-row panel, one FF2 partial per 128-wide hidden chunk
        # and the panel's arrival counter (the last chunk workgroup sums the partials and resets it)
        n_chunk = ff // 128 if (ff % 128 == 0 and d % 64 == 0 and d <= 256 and not glu) else 0
        self.mlp_part = z(((E + 31) // 32) * 32 * n_chunk * d) if n_chunk else None   # (16- or 32-row panels)
        self.mlp_cnt = z((E + 15) // 16, dt=i32) if n_chunk else None
        self.kv = [(z(E, H, Tmax, dh), z(E, H, Tmax, dh)) for _ in range(c.depth)]
        # decode weights (nn.Linear layouts; the GEMM operands are packed from them, self.wpk)
        self.w = dict(w_pin=z(d, S), act_emb=z(A, d) if not c.continuous else z(d, A),
                      act_emb_b=z(d) if c.continuous else None, reward_embed=z(d), w_se=z(d, S), b_se=z(d),
                      ln_final=z(d), w_h1=z(4 * d, c.in_dim), b_h1=z(4 * d), w_h2=z(nA + B, 4 * d),
                      b_h2=z(_r4(nA + B)), inv_freq=z(max(dh // 4, 1)), rs_mean=z(S + 1), rs_var=z(S + 1))
        self.nA = nA
        # k-major block-diagonal last head Linear (padding columns zero): the one-launch heads and the
        # row-resident step (xtrl_decode_step_rows, which also reads the k-major hidden layer)
        self.w['w_h2_t'] = z(4 * d, _r4(nA + B))
        self.rows_max = self._rows_max(c)
        self.row_part = self.row_cnt = None
        if self.rows_max:
            self.w['w_h1_t'] = z(c.in_dim, 4 * d)
            # its heads split over up to 4 workgroups per row: partial outputs and one counter per row
            self.row_part, self.row_cnt = z(E * 4 * _r4(nA + B)), z(E, dt=i32)
        # the one-launch heads (k_heads_mlp): split-bf16 image of the hidden layer, per 16-row panel one
        # partial output row block per 64-wide hidden chunk and an arrival counter
        if c.in_dim % 64 == 0 and d % 32 == 0:
            self.w['w_h1x'] = z(int(L.lib().xtrl_dgemm_packed_x6_elems(4 * d, c.in_dim)), dt=torch.int16)
            self.heads_part = z((E + 15) // 16 * (4 * d // 64) * 16 * _r4(nA + B))
            self.heads_cnt = z((E + 15) // 16, dt=i32)
        else:
            self.heads_part = self.heads_cnt = None
        self.w_lat = None
        self._pk_src = [(self.w, 'w_h1'), (self.w, 'w_h2')]
        self._alloc_body(z)
        # fragment-packed images of the decode GEMM weights (xtrl_dgemm_pack, refreshed by pack())
        pk = lambda t: z(int(L.lib().xtrl_dgemm_packed_floats(t.shape[0], t.shape[1])))
        self.wpk = {(id(src), k): pk(src[k]) for src, k in self._pk_src}
        self._build_desc(clamp, hazard_log2)
        self.graph = None

    def _alloc_body(self, z):
        """Per-layer decoder weights (self.wl) and their packed GEMM operands."""
        c = self.c
        d, I, ff = c.dim, c.inner, c.dim * c.ff_mult
        # w_out_t: to_out transposed for the attention kernel's fused out-projection
        f1 = 2 * ff if getattr(c, 'ff_glu', False) else ff   # (ff_glu: the GLU projection's value | gate rows)
        self.wl = [dict(ln_attn=z(d), w_qkv=z(self.n_qkv, d), b_qkv=z(_r4(self.n_qkv)), w_out=z(d, I), w_out_t=z(I, d),
                        ln_ff=z(d), w_ff1=z(f1, d), b_ff1=z(f1), w_ff2=z(d, ff), b_ff2=z(d)) for _ in range(c.depth)]
        if self.rows_max:   # k-major copies for the row-resident step
            for wl in self.wl:
                wl.update(w_qkv_t=z(d, _r4(self.n_qkv)), w_ff1_t=z(d, ff), w_ff2_t=z(ff, d))
        self._alloc_ff_images(z)
        self._pk_src += [(wl, k) for wl in self.wl for k in ('w_qkv', 'w_out', 'w_ff1', 'w_ff2')]

    def _alloc_ff_images(self, z):
        """FF1 / FF2 fragment images of the one-launch feed-forward kernel: the pre-split bf16 images
        (w_ff1x / w_ff2x, xtrl_dgemm_pack_x6) or, XTRL_MLP_IMG=f32, fp32 images (w_ff1f / w_ff2f,
        xtrl_dgemm_pack_f8: 2/3 of the bytes, the kernel splits each fragment before its MFMAs —
        measured slower: C3 rollout 23.3 vs 22.3 ms, C5 32.6 vs 31.4 ms; the split sits on the chain)."""
        c = self.c
        d, ff = c.dim, c.dim * c.ff_mult
        if not (ff % 128 == 0 and d % 64 == 0 and d <= 256) or getattr(c, 'ff_glu', False):
            return
        lib = L.lib()
        if os.environ.get('XTRL_MLP_IMG', 'x6') == 'x6':
            n1, n2 = (int(lib.xtrl_dgemm_packed_x6_elems(*s)) for s in ((ff, d), (d, ff)))
            for wl in self.wl:
                wl['w_ff1x'], wl['w_ff2x'] = z(n1, dt=torch.int16), z(n2, dt=torch.int16)
        else:
            n1, n2 = (int(lib.xtrl_dgemm_packed_f8_floats(*s)) for s in ((ff, d), (d, ff)))
            for wl in self.wl:
                wl['w_ff1f'], wl['w_ff2f'] = z(n1), z(n2)

    def _wv(self, src, k):
        """The tensor the descriptor points at for weight k of src: its packed image if it has one."""
        t = self.wpk.get((id(src), k), src.get(k))
        return L.ptr(t) if t is not None else None

    # ------------------------------------------------------------------------------------------
    def _build_desc(self, clamp, hazard_log2):
        c, Eg = self.c, self.E
        rows = L.ptr
        layers = (L.DecodeLayer * c.depth)()
        for i, (w, (kc, vc)) in enumerate(zip(self.wl, self.kv)):
            layers[i] = L.DecodeLayer(*(self._wv(w, k) for k in ('ln_attn', 'w_qkv', 'b_qkv', 'w_out', 'ln_ff', 'w_ff1',
                                                                 'b_ff1', 'w_ff2', 'b_ff2')), rows(kc), rows(vc),
                                      self._wv(w, 'w_out_t'), self._wv(w, 'w_ff1x'), self._wv(w, 'w_ff2x'),
                                      *(self._wv(w, k) for k in ('w_qkv_t', 'w_ff1_t', 'w_ff2_t', 'w_ff1f', 'w_ff2f')))
        D = L.DecodeDesc()
        D.E, D.S, D.A, D.B, D.d, D.L, D.H, D.dh, D.Tmax = (Eg, c.state_dim, c.num_actions, c.num_bins, c.dim,
                                                           c.depth, c.heads, c.dim_head, self.T)
        D.G, D.ff, D.in_dim, D.n_qkv = c.dim_gene, c.dim * c.ff_mult, c.in_dim, self.n_qkv
        D.continuous, D.squash, D.evolutionary = int(c.continuous), int(c.squash), int(c.evolutionary)
        D.gate_values, D.value_residual, D.learned_mix = int(c.gate_values), int(c.value_residual), int(c.learned_mix)
        D.rotary_abs, D.rot_dim = int(c.rotary_abs_rollout), c.dim_head // 2
        qk = bool(getattr(c, 'qk_norm', False))
        D.qk_norm, D.attn_scale = int(qk), float(c.qk_norm_scale) if qk else 0.
        D.xpos_base = float(c.xpos_scale_base) if getattr(c, 'rotary_xpos', False) else 0.
        D.rms_norm = int(getattr(c, 'rms_norm', False))
        D.sim_mode, D.hazard_log2, D.rs_eps = self.sim_mode, hazard_log2, 1e-5
        if clamp is not None:
            D.clamp_lo, D.clamp_hi, D.has_clamp = float(clamp[0]), float(clamp[1]), 1
        w = self.w
        for k in ('w_pin', 'b_pin', 'act_emb', 'act_emb_b', 'reward_embed', 'w_se', 'b_se', 'ln_final', 'w_h1', 'b_h1',
                  'w_h2', 'b_h2', 'inv_freq', 'rs_mean', 'rs_var', 'w_h1_t', 'w_h2_t', 'w_h1x'):
            setattr(D, k, self._wv(w, k))
        D.layers = C.cast(layers, C.POINTER(L.DecodeLayer))
        if self.rows_max:   # the row-resident step reads the layer descriptors from device memory
            raw = bytes(memoryview(layers).cast('B'))
            self._layers_dev = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.dev)
            D.layers_dev = C.cast(C.c_void_p(self._layers_dev.data_ptr()), C.POINTER(L.DecodeLayer))
        for k in ('state', 'prev_action', 'prev_action_f', 'prev_reward', 'alive', 'lens', 'cum_reward',
                  'episode_of_slot'):
            setattr(D, k, rows(getattr(self, k)))
        D.slot_of_row = None
        D.rng = self.rng.data_ptr()
        for k in ('states', 'actions', 'actions_f', 'logp', 'rewards', 'bounds', 'values'):
            setattr(D, 'traj_' + k, rows(self.traj[k]))
        for k in ('x', 'qkv', 'att', 'hff', 'ac_in', 'logits', 'v1', 'xn', 'live_rows', 'live_count', 'lat_embed',
                  'mlp_part', 'mlp_cnt', 'heads_part', 'heads_cnt', 'row_part', 'row_cnt', 'hglu'):
            setattr(D, k, rows(getattr(self, k)))
        D.ff_glu = int(self.hglu is not None)
        if os.environ.get('XTRL_DECODE_MLP', '1') == '0':   # A/B switch: the two-GEMM feed-forward
            D.mlp_part = None
        if os.environ.get('XTRL_DECODE_HEADS', '0') == '0':   # A/B switch: the one-launch heads (opt-in)
            D.heads_part = None
        self.desc, self._layers = D, layers

    # ------------------------------------------------------------------------------------------
    @torch.no_grad()
    def pack(self, model: WorldModelActorCritic, rs_mean, rs_var):
        """Copy (EMA) model weights into the decode layout (xtrl.py:721-734, 304-369 names)."""
        c, w = self.c, self.w
        w['w_pin'].copy_(model.transformer.project_in.weight)
        w['ln_final'].copy_(norm_gain(model.transformer.attn_layers.final_norm))
        inv = model.transformer.attn_layers.rotary_pos_emb.inv_freq
        w['inv_freq'][:inv.numel()].copy_(inv)
        self._pack_common(model, rs_mean, rs_var)
        I = c.inner
        for wl, (attn_l, ff_l) in zip(self.wl, model.blocks()):
            (ln_a, _, _), blk, _ = attn_l
            (ln_f, _, _), ffb, _ = ff_l
            wl['ln_attn'].copy_(norm_gain(ln_a))
            rows = [blk.to_q.weight, blk.to_k.weight, blk.to_v.weight]
            bias = [torch.zeros(3 * I, device=self.dev)]
            if blk.to_v_gate is not None:
                rows.append(blk.to_v_gate.weight)
                bias.append(blk.to_v_gate.bias)
            elif c.gate_values:
                raise RuntimeError('gate_values set but layer has no to_v_gate')
            if c.value_residual and c.learned_mix:
                if blk.to_value_residual_mix is not None:
                    rows.append(blk.to_value_residual_mix[0].weight)
                    bias.append(blk.to_value_residual_mix[0].bias)
                else:   # first layer: columns present but unused
                    rows.append(torch.zeros(c.heads, c.dim, device=self.dev))
                    bias.append(torch.zeros(c.heads, device=self.dev))
            torch.cat(rows, out=wl['w_qkv'])
            torch.cat(bias, out=wl['b_qkv'][:self.n_qkv])
            wl['w_out'].copy_(blk.to_out.weight)
            wl['w_out_t'].copy_(blk.to_out.weight.t())
            wl['ln_ff'].copy_(norm_gain(ln_f))
            f0 = ffb.ff[0].proj if c.ff_glu else ffb.ff[0][0]   # (ff_glu: the GLU projection)
            wl['w_ff1'].copy_(f0.weight)
            wl['w_ff2'].copy_(ffb.ff[2].weight)
            if f0.bias is not None:   # (ff_no_bias: the packed biases stay zero)
                wl['b_ff1'].copy_(f0.bias)
            if ffb.ff[2].bias is not None:
                wl['b_ff2'].copy_(ffb.ff[2].bias)
        self._pack_gemm_weights()

    def _pack_common(self, model, rs_mean, rs_var):
        """Action / reward / state embeddings, the actor-critic heads, RSNorm and the latent map —
        the parts every policy body shares (x_transformers_rl.py:304-369, fractal_rl.py:386-446)."""
        c, w = self.c, self.w
        if c.continuous:
            w['act_emb'].copy_(model.action_embeds.weight)
            w['act_emb_b'].copy_(model.action_embeds.bias)
        else:
            w['act_emb'].copy_(model.action_embeds.embed.weight)
        w['reward_embed'].copy_(model.reward_embed)
        w['w_se'].copy_(model.to_state_embed.weight)
        w['b_se'].copy_(model.to_state_embed.bias)
        torch.cat((model.action_head[0].weight, model.critic_head[0].weight), out=w['w_h1'])
        torch.cat((model.action_head[0].bias, model.critic_head[0].bias), out=w['b_h1'])
        # heads' last Linear as one block-diagonal weight over the [actor | critic] hidden row
        nA, d2 = self.nA, 2 * c.dim
        w['w_h2'].zero_()
        w['w_h2'][:nA, :d2].copy_(model.action_head[2].weight)
        w['w_h2'][nA:, d2:].copy_(model.critic_head[2].weight)
        torch.cat((model.action_head[2].bias, model.critic_head[2].bias), out=w['b_h2'][:nA + c.num_bins])
        w['rs_mean'].copy_(rs_mean)
        w['rs_var'].copy_(rs_var)
        if c.evolutionary:
            self.w_lat = (model.latent_to_embed.weight.detach().clone(), model.latent_to_embed.bias.detach().clone())

    def _pack_gemm_weights(self):
        w = self.w
        w['w_h2_t'][:, :w['w_h2'].shape[0]].copy_(w['w_h2'].t())
        if self.rows_max:   # k-major copies of the row-resident step
            w['w_h1_t'].copy_(w['w_h1'].t())
            for wl in self.wl:
                wl['w_qkv_t'][:, :self.n_qkv].copy_(wl['w_qkv'].t())
                wl['w_ff1_t'].copy_(wl['w_ff1'].t())
                wl['w_ff2_t'].copy_(wl['w_ff2'].t())
        lib = L.lib()
        if 'w_h1x' in w:
            t = w['w_h1']
            L.check(lib.xtrl_dgemm_pack_x6(L.ptr(t), t.shape[1], t.shape[0], t.shape[1], L.ptr(w['w_h1x']), L.stream()),
                    'dgemm_pack_x6(w_h1)')
        for src, k in self._pk_src:
            t = src[k]
            L.check(lib.xtrl_dgemm_pack(L.ptr(t), t.shape[1], t.shape[0], t.shape[1], L.ptr(self.wpk[(id(src), k)]),
                                        L.stream()), f'dgemm_pack({k})')
        for wl in getattr(self, 'wl', ()):
            for src, dst in (('w_ff1', 'w_ff1x'), ('w_ff2', 'w_ff2x')):
                if dst in wl:
                    t = wl[src]
                    L.check(lib.xtrl_dgemm_pack_x6(L.ptr(t), t.shape[1], t.shape[0], t.shape[1], L.ptr(wl[dst]),
                                                   L.stream()), f'dgemm_pack_x6({src})')
            for src, dst in (('w_ff1', 'w_ff1f'), ('w_ff2', 'w_ff2f')):
                if dst in wl:
                    t = wl[src]
                    L.check(lib.xtrl_dgemm_pack_f8(L.ptr(t), t.shape[1], t.shape[0], t.shape[1], L.ptr(wl[dst]),
                                                   L.stream()), f'dgemm_pack_f8({src})')

    # ------------------------------------------------------------------------------------------
    def _begin(self, seed, update, slot_offset, episode_of_slot, latent, slots=None):
        """``slots``: per-row global pair indices keying the sampling stream (gene-sharded ranks);
        None: rows are the contiguous pairs slot_offset, slot_offset + 1, ..."""
        # the small per-rollout uploads (rng words, slots, episode ids) through one pinned stage and
        # asynchronous copies: a pageable upload blocks the host (host-env waves begin every episode)
        E = self.E
        st = getattr(self, '_begin_stage', None)
        if st is None:
            st = self._begin_stage = torch.empty(4 + 2 * E, dtype=torch.int32, pin_memory=True)
            self._begin_np = st.numpy()
            self._begin_done = torch.cuda.Event()
        else:
            self._begin_done.synchronize()   # (the previous rollout's copies out of the stage are done)
        a = self._begin_np
        a[:4].view(np.int64)[:] = (seed & 0x7FFFFFFFFFFFFFFF, (int(update) & 0xFFFFFFFF) | (int(slot_offset) << 32))
        self.rng.copy_(st[:4].view(torch.int64), non_blocking=True)
        if slots is not None:
            a[4:4 + E] = slots
            self.slot_of_row.copy_(st[4:4 + E], non_blocking=True)
        self.desc.slot_of_row = self.slot_of_row.data_ptr() if slots is not None else None
        if episode_of_slot.is_cuda:
            self.episode_of_slot.copy_(episode_of_slot.to(torch.int32))
        else:
            a[4 + E:4 + 2 * E] = episode_of_slot.numpy()
            self.episode_of_slot.copy_(st[4 + E:4 + 2 * E], non_blocking=True)
        self._begin_done.record()
        torch._foreach_zero_([t for t in self.traj.values() if t is not None])
        if self.c.evolutionary:
            self.lat_embed.copy_(F.linear(latent, *self.w_lat))
        L.check(L.lib().xtrl_rollout_begin(C.byref(self.desc), L.stream()), 'rollout_begin')

    # the row-resident decode step (xtrl_decode_step_rows) takes over once at most this many rows are
    # live: for d <= 128 a row's weights (<= ~2 MB) stream from the XCD's L2 and one launch per step
    # beats the ~15 dependent launches of the multi-kernel step up to one workgroup per CU; wider
    # models keep the multi-kernel step (their weights outgrow the L2).  XTRL_DECODE_ROWS=0: off.
    ROWS = True

    def _rows_max(self, c):
        if not self.ROWS or os.environ.get('XTRL_DECODE_ROWS', '1') == '0':
            return 0
        nA = 2 * c.num_actions if c.continuous else c.num_actions
        if (c.dim > 128 or c.depth > 8 or nA > 64 or self.E > 8192 or (c.dim * c.ff_mult) % 4
                or getattr(c, 'ff_glu', False)):
            return 0
        r4 = lambda x: (x + 3) & ~3
        d, I, ff = c.dim, c.heads * c.dim_head, c.dim * c.ff_mult   # decode.hip row_lds (in_dim <= 3 d)
        lds = (2 * r4(d) + r4(self.n_qkv) + 2 * r4(I) + r4(max(ff, 4 * d)) + 3 * d + 4096 + r4(nA + c.num_bins)
               + c.heads * (r4(self.T) + 64) + 64)
        return 256 if 4 * lds <= 96 * 1024 else 0

    def step(self, t, rows=False):
        """Decode step t: the multi-kernel step, or (``rows``) the row-resident one."""
        if rows:
            L.check(L.lib().xtrl_decode_step_rows(C.byref(self.desc), int(t), self.rows_max, L.stream()),
                    f'decode_step_rows(t={t})')
            return
        L.check(L.lib().xtrl_decode_step(C.byref(self.desc), int(t), L.stream()), f'decode_step(t={t})')

    def _steps(self):
        rows = 0 < self.E <= self.rows_max
        for t in range(self.T):
            self.step(t, rows)

    def cache_tensors(self):
        """The per-episode decode state carried between deploy calls (Agent.forward hiddens)."""
        return [t for kv in self.kv for t in kv] + [self.v1]

    CHUNK = int(os.environ.get('XTRL_ROLLOUT_CHUNK', '32'))   # steps per captured sub-graph

    @torch.no_grad()
    def run(self, seed, update, episode_of_slot, latent=None, slot_offset=0, slots=None):
        """Roll out Tmax steps of the device Sim for all E slots; returns the trajectory dict.

        Graph mode: the T steps are captured as sub-graphs of CHUNK steps.  After launching chunk i
        the host waits for chunk i - 1 (the GPU meanwhile runs chunk i) and reads the live-row count
        of its last step (copied to pinned memory inside the stream); once a chunk ended with no
        live episode, no further chunk is launched — the dead tail of a long-T rollout (C2: T = 500,
        the longest of 768 episodes ~425 steps at hazard 1/64) costs one chunk, not T - max_len steps."""
        assert self.sim_mode != SIM_HOST
        self._begin(seed, update, slot_offset, episode_of_slot, latent, slots)
        if not self.use_graph:
            self._steps()
            self._clear_end_markers()
            return self.traj
        if self.graph is None:
            self._steps()   # warm-up launch outside capture (code objects loaded)
            if self.rows_max and self.E > self.rows_max:
                self._begin(seed, update, slot_offset, episode_of_slot, latent, slots)
                for t in range(self.T):
                    self.step(t, True)   # (the row-resident kernel's code object too)
            self._begin(seed, update, slot_offset, episode_of_slot, latent, slots)
            CH = max(1, self.CHUNK)
            self._chunks = [(t0, min(t0 + CH, self.T)) for t0 in range(0, self.T, CH)]
            self._live_host = torch.zeros(len(self._chunks), dtype=torch.int32, pin_memory=True)
            self._live_dev = torch.zeros(len(self._chunks), dtype=torch.int32, device=self.dev)
            # two graph sets: the multi-kernel step, and (rows_max) the row-resident step for the chunks
            # after the live count has dropped to rows_max (it never rises within a rollout)
            graphs = {}
            for rows in [False] + ([True] if self.rows_max else []):
                graphs[rows] = []
                for i, (t0, t1) in enumerate(self._chunks):
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        for t in range(t0, t1):
                            self.step(t, rows)
                        # live rows at the chunk's last step (its compaction counted them)
                        self._live_dev[i:i + 1].copy_(self.live_count[(t1 - 1) & 1:((t1 - 1) & 1) + 1])
                    graphs[rows].append(g)
            self.graph = graphs
            self._chunk_ev = [torch.cuda.Event() for _ in self._chunks]
        stream = torch.cuda.current_stream()
        rows = 0 < self.E <= self.rows_max
        self.chunks_rows = 0
        self.rows_from_step = 0 if rows else self.T   # first step decoded by the row-resident step
        for i in range(len(self._chunks)):
            if rows and self.rows_from_step == self.T:
                self.rows_from_step = self._chunks[i][0]
            self.graph[rows][i].replay()
            self.chunks_rows += int(rows)
            self._live_host[i:i + 1].copy_(self._live_dev[i:i + 1], non_blocking=True)
            self._chunk_ev[i].record(stream)
            if i >= 1:
                self._chunk_ev[i - 1].synchronize()
                live = int(self._live_host[i - 1])
                if live == 0:
                    break
                rows = rows or live <= self.rows_max
        self._clear_end_markers()
        return self.traj

    def _clear_end_markers(self):
        """The row-resident step marks a row it ended with alive = ALIVE_END + (t & 1) (3 / 4, live for
        the rest of that launch; csrc/decode.hip ``live_at``) and the next step's compaction clears it.
        After the rollout's last step no compaction follows: clear them here so ``alive`` leaves the
        rollout with 0 = dead, 1 = live only (no host sync: two stream-ordered ops)."""
        self.alive.mul_(self.alive.lt(3))

    def _host_decode(self, t, rows_max, desc, act_p, stream):
        """Decode step t of a host-env wave, its actions to the pinned buffer, one host wait."""
        L.check(L.lib().xtrl_host_decode(desc, t, rows_max, act_p, stream), f'host_decode(t={t})')

    @torch.no_grad()
    def run_host_wave(self, env_reset, env_step, seed, update, rows, latent=None, slots=None, max_steps=None,
                      bootstrap=True):
        """One wave of a host-env rollout (xtrl.py:1232-1341) over this engine's E rows, the first
        ``rows`` of them live (a partial last wave leaves the rest dead).  ``env_reset() -> [E][S]``,
        ``env_step(actions, live) -> (next_state [E][S], reward [E], terminated [E], truncated [E])``
        as numpy (``actions``: int [E] or float [E][A]; ``live``: bool [E] mask of rows whose
        episode is running).  Per step one device->host copy of the actions and one host->device
        copy of the env results.  The engine holds Tmax = max_timesteps + 1 positions so a
        truncation at the last step can still take its bootstrap decode step.
        Returns (traj, lens [E] host int, totals [E] host float64, boot_rows)."""
        assert self.sim_mode == SIM_HOST
        import numpy as np
        E, S, A = self.E, self.c.state_dim, self.c.num_actions
        T = min(self.T - 1, max_steps or self.T - 1)
        if getattr(self, '_host_stage', None) is None:
            self._host_stage = torch.empty(E * (S + 1) + 2 * E, dtype=torch.float32, pin_memory=True)
            self._host_act = torch.empty(E * (A if self.c.continuous else 1),
                                         dtype=torch.float32 if self.c.continuous else torch.int32, pin_memory=True)
        # zero copy both ways: the sampling stores the actions into the pinned buffer itself and the
        # feedback kernel reads the pinned stage in place (dev_stage NULL)
        self.desc.act_host = self._host_act.data_ptr()
        st = self._host_stage
        state0 = np.asarray(env_reset(), dtype=np.float32).reshape(E, S)
        # (through the pinned stage, asynchronously: the stage's state rows are next written after the
        #  first decode step has completed)
        st[:E * S].numpy()[:] = state0.reshape(-1)
        self.state.copy_(st[:E * S].view(E, S), non_blocking=True)
        eps = getattr(self, '_host_eps', None)
        if eps is None:
            eps = self._host_eps = torch.arange(E, dtype=torch.int32)
        self._begin(seed, update, 0, eps, latent, slots)
        live = np.arange(E) < rows
        if rows < E:
            self.alive[rows:].zero_()
        boot_rows = np.zeros(E, dtype=bool)
        lens = np.zeros(E, dtype=np.int64)
        totals = np.zeros(E, dtype=np.float64)
        lib = L.lib()
        st_state = st[:E * S].view(E, S).numpy()
        st_rew, st_flags = st[E * S:E * (S + 1)].numpy(), st[E * (S + 1):].view(torch.uint8)
        flags = st_flags.numpy()
        act_np = self._host_act.numpy().reshape(E, A) if self.c.continuous else self._host_act.numpy()
        # one library call per half step: decode + action copy + the step's one host wait, then the
        # env's results staged back + the feedback kernel (xtrl_host_decode / xtrl_host_feedback)
        desc, stream = C.byref(self.desc), L.stream()
        act_p, st_p, dst_p = self._host_act.data_ptr(), st.data_ptr(), None
        rows_max = self.rows_max if 0 < E <= self.rows_max else 0
        pending = np.zeros(E, dtype=bool)    # rows taking their bootstrap decode step
        # host-side time of the wave's steps (seconds): decode launch + the step's wait for the actions,
        # the env step, the feedback (staging + H2D copy + kernel launch) — bench.py reports them
        ht = self.host_times = dict(decode=0., env=0., feedback=0., steps=0)
        clock = time.perf_counter

        def env_half(t, c1):
            """The env step on step t's actions and its results staged (pinned); lens / totals / live /
            pending bookkeeping.  Returns the staging end time."""
            nonlocal live, pending
            pending[:] = False
            ns, r, term, trunc = env_step(act_np, live.copy())
            c2 = clock()
            ns = np.asarray(ns, dtype=np.float32).reshape(E, S)
            r = np.asarray(r, dtype=np.float64).reshape(E)
            term = np.asarray(term).reshape(E).astype(bool)
            trunc = np.asarray(trunc).reshape(E).astype(bool)
            totals[live] += r[live]
            lens[live] = t + 1
            st_state[:] = ns
            st_rew[:] = r
            flags[:E] = term
            flags[E:2 * E] = trunc
            ht['env'] += c2 - c1
            ended = live & (term | trunc | (t + 1 >= T))
            boot_now = live & trunc & ~term & bool(bootstrap)     # the last step (t + 1 == T) included
            boot_rows[:] |= boot_now
            pending = boot_now
            live = live & ~ended
            return clock()

        scalar_step = getattr(env_step, 'scalar', None)

        def env_half1(t, c1):
            """env_half for one row of a scalar env (the reference contract) on Python scalars: the
            same staging and bookkeeping without the per-step numpy temporaries (~10 us a step)."""
            a = act_np[0].tolist() if self.c.continuous else int(act_np[0])
            ns, r, term, trunc = scalar_step(a)
            c2 = clock()
            r, term, trunc = float(np.asarray(r, dtype=np.float64).reshape(-1)[0]), bool(term), bool(trunc)
            st_state[0] = np.asarray(ns, dtype=np.float32).reshape(S)
            st_rew[0] = r
            flags[0] = term
            flags[1] = trunc
            ht['env'] += c2 - c1
            was = bool(live[0])
            if was:
                totals[0] += r
                lens[0] = t + 1
            boot = was and trunc and not term and bool(bootstrap)
            if boot:
                boot_rows[0] = True
            pending[0] = boot
            if was and (term or trunc or t + 1 >= T):
                live[0] = False
            return clock()

        t0 = 0
        if E == 1 and rows_max > 0 and os.environ.get('XTRL_HOST_GATE', '1') != '0':
            t0 = self._run_host_gated(T, bootstrap, desc, stream, st_p, dst_p,
                                      env_half1 if scalar_step is not None else env_half, lambda: live,
                                      lambda: pending)
        for t in range(t0, T + 1):
            if not live.any() and not pending.any():
                break
            if not live.any():   # only bootstrap rows: their decode step, no env step
                self.step(t, rows_max > 0)
                self.alive.zero_()   # (the row-resident step leaves them at 2 for a feedback that never comes)
                break
            c0 = clock()
            self._host_decode(t, rows_max, desc, act_p, stream)
            c1 = clock()
            c2 = env_half(t, c1)
            L.check(lib.xtrl_host_feedback(desc, t, st_p, dst_p, T, int(bootstrap), stream), 'host_feedback')
            c3 = clock()
            ht['decode'] += c1 - c0
            ht['feedback'] += c3 - c2
            ht['steps'] += 1
        torch.cuda.current_stream().synchronize()   # the pinned staging buffer is reused next wave
        return self.traj, lens, totals, boot_rows

    HOST_GATE_AHEAD = 2   # gated steps queued ahead of the host (one decode in flight, the next waiting)

    def _run_host_gated(self, T, bootstrap, desc, stream, st_p, dst_p, env_half, live_of, pending_of):
        """The scalar-env wave (E == 1) on gated steps (xtrl_host_row_step): each decode launch is
        queued ahead and waits on the device for the host's go, applies the previous env step's
        results from the pinned stage itself, and publishes its completion in pinned memory — no
        launch, stream synchronisation or feedback launch between an env step and the next decode.
        Returns the step from which the ungated loop continues (T + 1: the wave is done)."""
        lib = L.lib()
        if getattr(self, '_host_gate', None) is None:
            self._host_gate = torch.zeros(3, dtype=torch.int32, pin_memory=True)   # go | done | gave up
        g = self._host_gate.numpy()
        gate_p = self._host_gate.data_ptr()
        done_p = gate_p + 4
        g[:] = 0
        ht, clock = self.host_times, time.perf_counter

        def enqueue(t):
            L.check(lib.xtrl_host_row_step(desc, t, st_p, T, int(bootstrap), gate_p, stream), f'host_row_step(t={t})')

        def wait(v):
            rc = lib.xtrl_host_wait(done_p, v, 120.0)
            if rc < 0:
                g[0] = -1
                raise RuntimeError(f'host_row_step: step {v - 1} did not complete')
            return rc == 0

        nxt = 0
        while nxt < min(self.HOST_GATE_AHEAD, T + 1):
            enqueue(nxt)
            nxt += 1
        resume = T + 1
        t = 0
        g[0] = 1   # go: step 0 (no env results yet)
        try:
            while True:
                c0 = clock()
                if nxt <= T:   # (queued while the device runs step t)
                    enqueue(nxt)
                    nxt += 1
                if not wait(t + 1):   # the device gave up waiting: steps t - 1's results unapplied, t not run
                    resume = t
                    break
                c1 = clock()
                c2 = env_half(t, c1)
                ht['decode'] += c1 - c0
                ht['steps'] += 1
                g[0] = t + 2   # go: step t + 1 (it applies step t's results first)
                ht['feedback'] += clock() - c2
                if not live_of().any():   # step t + 1 only applies the results (and decodes a bootstrap row)
                    if not wait(t + 2):
                        resume = t + 1
                    elif pending_of().any():
                        self.alive.zero_()   # (the bootstrap step leaves alive 2 for a feedback that never comes)
                    break
                t += 1
        except BaseException:
            g[0] = -1   # an env that raised (or an interrupt): release the queued steps at once, and
            torch.cuda.current_stream().synchronize()   # let them drain before the gate is reused
            raise
        g[0] = -1   # cancel the steps still queued
        torch.cuda.current_stream().synchronize()
        if resume <= T and resume > 0:   # the ungated loop resumes at `resume`: its previous results first
            L.check(lib.xtrl_host_feedback(desc, resume - 1, st_p, dst_p, T, int(bootstrap), stream), 'host_feedback')
        return resume


class FractalRolloutEngine(RolloutEngine):
    """KV-cached rollout of the causal fractal policy body (fractal.FractalPolicyActorCritic)
    through ``xtrl_fractal_decode_step``.  Per level it keeps the self-attention K/V caches and the
    running sum of the level's outputs over the episode so far (the causal mean pools of the
    global-state update and the level projection); the step's global state starts at
    global_state_init and is updated level by level (fractal_rl.py:318-340, causal)."""

    ROWS = False   # (no row-resident form of the fractal step)

    def _host_decode(self, t, rows_max, desc, act_p, stream):
        self.step(t)
        src = self.prev_action_f if self.c.continuous else self.prev_action
        self._host_act.copy_(src.reshape(-1), non_blocking=True)
        torch.cuda.current_stream().synchronize()

    def __init__(self, model, E: int, Tmax: int, **kw):
        c = dataclasses.replace(model.cfg, depth=model.levels, gate_values=False, value_residual=False,
                                learned_mix=False, rotary_abs_rollout=False)
        self.levels = model.levels
        self.ln_eps = float(model.fractal_encoder.get_fractal_block(0).norm1.eps)
        super().__init__(model, E, Tmax, cfg=c, **kw)

    def _alloc_body(self, z):
        c, E, Lv = self.c, self.E, self.levels
        d, I, ff = c.dim, c.inner, c.dim * c.ff_mult
        # g_init / g carry d zero columns after the state: the fused global-update | level-projection
        # GEMM's residual reads them for its projection half (include/xtrl_hip.h XtrlFractalDesc)
        self.w.update(b_pin=z(d), g_init=z(2 * d), c0=z(d), w_fa0=z(2 * d, (Lv + 1) * d), b_fa0=z(2 * d),
                      w_fa2=z(d, 2 * d), b_fa2=z(d))
        # w_out_t: to_out transposed for the attention kernel's fused out-projection + post-norms
        self.wl = [dict(w_qkv=z(3 * I, d), w_out=z(d, I), w_out_t=z(I, d), ln1_w=z(d), ln1_b=z(d), w_c=z(d, d),
                        ln2_w=z(d), ln2_b=z(d),
                        w_ff1=z(ff, d), b_ff1=z(ff), w_ff2=z(d, ff), b_ff2=z(d), ln3_w=z(d), ln3_b=z(d),
                        w_pg=z(2 * d, d), b_pg=z(2 * d), level_emb=z(d), sums=z(E, d)) for _ in range(Lv)]
        self._alloc_ff_images(z)   # fragment images for the one-launch feed-forward
        self.fbuf = dict(g=z(E, 2 * d), c2=z(E, d), tmp=z(E, d), x2=z(E, d), mean=z(E, d), allf=z(E, (Lv + 1) * d),
                         hagg=z(E, 2 * d))
        self._pk_src += [(self.w, k) for k in ('w_fa0', 'w_fa2')]
        self._pk_src += [(wl, k) for wl in self.wl for k in ('w_qkv', 'w_out', 'w_c', 'w_ff1', 'w_ff2', 'w_pg')]

    def _build_desc(self, clamp, hazard_log2):
        super()._build_desc(clamp, hazard_log2)
        self.desc.state_only = 1
        Lv = self.levels
        levels = (L.FractalLevel * Lv)()
        names = [n for n, _ in L.FractalLevel._fields_]
        for i, wl in enumerate(self.wl):
            levels[i] = L.FractalLevel(*(self._wv(wl, k) for k in names))
        F_ = L.FractalDesc()
        F_.levels, F_.ln_eps = Lv, self.ln_eps
        F_.level = C.cast(levels, C.POINTER(L.FractalLevel))
        for k in ('g_init', 'c0', 'w_fa0', 'b_fa0', 'w_fa2', 'b_fa2'):
            setattr(F_, k, self._wv(self.w, k))
        for k, t in self.fbuf.items():
            setattr(F_, k, L.ptr(t))
        self.fdesc, self._flevels = F_, levels

    @torch.no_grad()
    def pack(self, model, rs_mean, rs_var):
        """Copy the (EMA) fractal body into the decode layout (fractal_rl.py:274-346 names)."""
        w = self.w
        enc = model.fractal_encoder
        w['w_pin'].copy_(enc.input_embed.weight)
        w['b_pin'].copy_(enc.input_embed.bias + model.level_embed(0))   # level 0's embedding folded in
        self._pack_common(model, rs_mean, rs_var)
        d = self.c.dim
        w['g_init'][:d].copy_(enc.global_state_init.reshape(-1))
        gu = enc.global_state_update
        fa0, fa2 = enc.final_aggregation[0], enc.final_aggregation[2]
        w['w_fa0'].copy_(fa0.weight)
        w['b_fa0'].copy_(fa0.bias)
        w['w_fa2'].copy_(fa2.weight)
        w['b_fa2'].copy_(fa2.bias)
        for li, wl in enumerate(self.wl):
            blk = enc.get_fractal_block(li)
            sa, ga = blk.self_attn, blk.global_attn
            torch.cat((sa.to_q.weight, sa.to_k.weight, sa.to_v.weight), out=wl['w_qkv'])
            wl['w_out'].copy_(sa.to_out.weight)
            wl['w_out_t'].copy_(sa.to_out.weight.t())
            # the one-key cross-attention W_out (W_v g) as one operand W_c = W_out W_v (library GEMM)
            ops.gemm(ga.to_out.weight, ga.to_v.weight.t().contiguous(), out=wl['w_c'])
            for j, nm in ((1, blk.norm1), (2, blk.norm2), (3, blk.norm3)):
                wl[f'ln{j}_w'].copy_(nm.weight)
                wl[f'ln{j}_b'].copy_(nm.bias)
            ff0, ff2 = blk.ff.ff[0][0], blk.ff.ff[2]
            wl['w_ff1'].copy_(ff0.weight)
            wl['b_ff1'].copy_(ff0.bias)
            wl['w_ff2'].copy_(ff2.weight)
            wl['b_ff2'].copy_(ff2.bias)
            pj = enc.level_projections[li]
            torch.cat((gu.weight, pj.weight), out=wl['w_pg'])
            torch.cat((gu.bias, pj.bias), out=wl['b_pg'])
            wl['level_emb'].copy_(model.level_embed(li))
        # level 0's cross-attention row: every row's global state is global_state_init there
        ops.gemm(w['g_init'][None, :d], self.wl[0]['w_c'], out=w['c0'][None])
        self._pack_gemm_weights()

    def step(self, t, rows=False):
        L.check(L.lib().xtrl_fractal_decode_step(C.byref(self.desc), C.byref(self.fdesc), int(t), L.stream()),
                f'fractal_decode_step(t={t})')

    def cache_tensors(self):
        return [t for kv in self.kv for t in kv] + [wl['sums'] for wl in self.wl]


def make_engine(model, E, Tmax, **kw):
    """The rollout engine of a policy body: the decoder's or the fractal body's."""
    cls = FractalRolloutEngine if getattr(model, 'levels', None) is not None else RolloutEngine
    return cls(model, E, Tmax, **kw)
