"""Learner / Agent with the reference API (x_transformers_rl.py:644-1380), MI355X-native inside.

    learner = Learner(state_dim, num_actions, reward_range, world_model=dict(...), ...)
    learner(env, num_learning_updates, seed=None, max_timesteps=None)
    raw_actions, hiddens = learner.agent(state, reward=None, hiddens=None, latent_gene_id=0)

Environments
  * ``SynthVecSim`` (or anything with ``xtrl_device_sim = True``): the synthetic LunarLander-shaped
    Sim runs on the device inside the rollout step; all (episode, gene) pairs of an update are
    rolled out as one vectorised batch (the reference runs them one by one, xtrl.py:1220).
  * any reference-style env (``reset(seed=?) -> state | (state, ...)``, ``step(action) ->
    (state, reward, terminated[, truncated, ...])``, xtrl.py:1232-1305): episodes are rolled
    out one at a time with batch 1, exactly like the reference loop, the policy step still on
    the device.
  * a vectorised host env (``num_envs`` sub-envs, batched reset / step): the pairs run in waves
    of num_envs through the same batched decode (``Learner.rollout_host``).

Randomness protocol (shared with the oracle, see oracle/ref_port.py):
  sampling uniforms  philox(seed; slot, t, update, FIELD_SAMPLE)   slot = global pair index
  minibatch order    torch.randperm with a generator seeded from (seed, update, epoch)
  reward-drop coin   philox(seed; minibatch, epoch, update, FIELD_COIN)
  EPO evolve_        private generator seeded from (seed, update, epoch, minibatch)
"""
from __future__ import annotations

import copy
import math
import os
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from . import _lib as L
from . import distributed as dist_
from . import ops
from .evolution import LatentGenePool, evolve_seed
from .model import ModelConfig, WorldModelActorCritic
from .params import FlatParams
from .fractal import FractalPolicyActorCritic
from .rollout import SIM_HOST, SIM_LANDER, SIM_README, make_engine
from .train import rsnorm_update


# ema-pytorch EMA keyword defaults the restatement honours (xtrl.py:747 passes **ema_kwargs)
EMA_DEFAULTS = dict(update_after_step=100, update_every=10, inv_gamma=1., power=2 / 3, min_value=0.,
                    update_model_with_ema_every=None, update_model_with_ema_beta=0.)


# x-transformers Decoder / Attention / FeedForward options (>= 2.3, the reference's pin, pyproject.toml:35)
# at their default values: passing one of them explicitly builds the network the MI355X decoder runs
XT_DEFAULTS = dict(
    cross_attend=False, only_cross=False, use_scalenorm=False, use_rmsnorm=False, use_simple_rmsnorm=False,
    alibi_pos_bias=False, rel_pos_bias=False, dynamic_pos_bias=False, rotary_xpos=False, residual_attn=False,
    cross_residual_attn=False, macaron=False, pre_norm=True, gate_residual=False, scale_residual=False,
    shift_tokens=0, sandwich_norm=False, resi_dual=False, zero_init_branch_output=False, layer_dropout=0.,
    use_layerscale=False, unet_skips=False, reinject_input=False, weight_tie_layers=False,
    ff_glu=False, ff_swish=False, ff_relu_squared=False, ff_post_act_ln=False, ff_no_bias=False,
    attn_talking_heads=False, attn_head_scale=False, attn_sparse_topk=None, attn_num_mem_kv=0, attn_on_attn=False,
    attn_gate_value_heads=False, attn_swiglu_values=False, attn_qk_norm=False, attn_one_kv_head=False,
    attn_kv_heads=None, attn_shared_kv=False, attn_value_dim_head=None, attn_add_zero_kv=False,
    attn_rotary_embed_values=False, attn_max_attend_past=None)


def epoch_permutation(seed, update, epoch, n):
    g = torch.Generator().manual_seed((int(seed) * 1000003 + int(update)) * 1000003 + int(epoch) & (2 ** 62 - 1))
    return torch.randperm(n, generator=g)


def reward_coin(seed, update, epoch, minibatch, p):
    if p <= 0.:
        return True
    u = L.rng_uniform(int(seed), int(update), int(minibatch), int(epoch), L.FIELD_COIN, 0)
    return bool(np.float32(u) >= np.float32(p))


class SynthVecSim:
    """Descriptor of the device-resident synthetic Sim (csrc/philox.h, oracle/philox.py):
    'lander': S-dim N(0,1) states, reward N(0,1) * (1 + 0.1 a), termination hazard 2^-hazard_log2;
    'readme': the README Sim (N(0,1) states and rewards, never terminates)."""

    xtrl_device_sim = True

    def __init__(self, state_dim, num_actions, mode='lander', hazard_log2=6):
        assert mode in ('lander', 'readme')
        self.state_dim, self.num_actions, self.mode, self.hazard_log2 = state_dim, num_actions, mode, hazard_log2


# ----------------------------------------------------------------------------------------------
# Agent (xtrl.py:644-1065)
# ----------------------------------------------------------------------------------------------


class Agent(nn.Module):
    def __init__(self, state_dim, num_actions, reward_range, epochs, max_timesteps, batch_size, lr, betas, lam,
                 gamma, beta_s, regen_reg_rate, cautious_factor, eps_clip, value_clip, ema_decay,
                 continuous_actions=False, squash_continuous=True, critic_pred_num_bins=100, hidden_dim=48,
                 evolutionary=False, evolve_every=1, evolve_after_step=20,
                 latent_gene_pool: dict = dict(dim=128, num_genes_per_island=3, num_selected=2, tournament_size=2),
                 world_model: dict = dict(attn_dim_head=16, heads=4, depth=4, attn_gate_values=True,
                                          add_value_residual=True, learned_value_residual_mix=True),
                 dropout=0.25, max_grad_norm=0.5, frac_actor_critic_head_gradient=0.5,
                 ema_kwargs: dict = dict(update_model_with_ema_every=1250), save_path='./ppo.pt', accelerator=None,
                 actor_loss_weight=1., critic_loss_weight=1., autoregressive_loss_weight=1.,
                 # extensions (decision log in DESIGN.md)
                 reward_dropout=0.5, seed=0, rotary_abs_rollout=False, hl_reduction_mean=True, hl_sigma_ratio=2.0,
                 fused_learn=True, device=None, truncation_bootstrap=True, policy_body='decoder', fractal_levels=None,
                 packed_learn=False):
        super().__init__()
        self.accelerator = accelerator if accelerator is not None else dist_.DistContext(device)
        dev = self.accelerator.device
        wm = dict(world_model)
        # x-transformers switches that select an implementation, not the math: accepted and ignored
        # (attn_flash: fused scaled-dot-product attention instead of the explicit softmax — the same
        # function; attn_onnxable: an export-friendly softmax; the learn step's attention here is always
        # the fused HIP kernel).  Options given at their x-transformers default build the same network:
        # accepted too.
        for k in ('attn_flash', 'attn_onnxable'):
            wm.pop(k, None)
        # x-transformers' Decoder refuses an explicit causal flag (it always is causal)
        assert 'causal' not in wm, 'cannot set causality on decoder'
        for k, default in XT_DEFAULTS.items():
            if k in wm and wm[k] == default:
                wm.pop(k)
        known = {'attn_dim_head', 'heads', 'depth', 'attn_gate_values', 'add_value_residual',
                 'learned_value_residual_mix', 'ff_mult', 'ff_no_bias', 'ff_glu', 'attn_qk_norm',
                 'attn_qk_norm_scale', 'rotary_xpos', 'rotary_xpos_scale_base', 'use_rmsnorm'}
        unknown = set(wm) - known
        if unknown:
            raise NotImplementedError(f'world_model options {sorted(unknown)} are not supported by the MI355X decoder '
                                      f'(supported: {sorted(known)}, implementation switches attn_flash / '
                                      f'attn_onnxable, and any option at its x-transformers default)')
        self.seed = int(seed)
        self.evolutionary = evolutionary
        self.evolve_every, self.evolve_after_step = evolve_every, evolve_after_step
        self.gene_pool = LatentGenePool(**latent_gene_pool) if evolutionary else None
        c = ModelConfig(state_dim=state_dim, num_actions=num_actions, dim=hidden_dim, depth=wm.get('depth', 1),
                        heads=wm.get('heads', 8), dim_head=wm.get('attn_dim_head', 64), num_bins=critic_pred_num_bins,
                        reward_range=tuple(reward_range), continuous=continuous_actions, squash=squash_continuous,
                        evolutionary=evolutionary, dim_gene=self.gene_pool.dim_gene if evolutionary else 0,
                        frac_head_grad=frac_actor_critic_head_gradient, entropy_weight=beta_s, eps_clip=eps_clip,
                        value_clip=value_clip, dropout=dropout, reward_dropout=reward_dropout,
                        gate_values=wm.get('attn_gate_values', False), value_residual=wm.get('add_value_residual', False),
                        learned_mix=wm.get('learned_value_residual_mix', False), ff_mult=int(wm.get('ff_mult', 4)),
                        ff_no_bias=bool(wm.get('ff_no_bias', False)), ff_glu=bool(wm.get('ff_glu', False)),
                        rms_norm=bool(wm.get('use_rmsnorm', False)), qk_norm=bool(wm.get('attn_qk_norm', False)),
                        qk_norm_scale=float(wm.get('attn_qk_norm_scale', 10.)),
                        rotary_xpos=bool(wm.get('rotary_xpos', False)),
                        xpos_scale_base=float(wm.get('rotary_xpos_scale_base', 512.)),
                        rotary_abs_rollout=rotary_abs_rollout,
                        hl_reduction_mean=hl_reduction_mean, hl_sigma_ratio=hl_sigma_ratio)
        self.cfg = c
        # the learn step without the minibatch's padding (XtrlTrainDesc.packed): exact only with the
        # per-token critic reduction, where no loss term or gradient involves a padded token
        if packed_learn and (hl_reduction_mean or not fused_learn or policy_body != 'decoder'):
            raise ValueError('packed_learn needs hl_reduction_mean=False, fused_learn=True and the decoder policy body: '
                             'with the scalar HL-Gauss mean the padded tokens carry critic gradient')
        self.packed_learn = bool(packed_learn)
        # policy body: the x-transformers Decoder (x_transformers_rl.py) or the per-timestep causal
        # fractal encoder (fractal_rl.py:349-619 made causal, fractal.FractalPolicyActorCritic)
        if policy_body == 'fractal':
            if c.gate_values or c.value_residual or c.ff_no_bias or c.ff_glu or c.qk_norm or c.rotary_xpos or c.rms_norm:
                raise NotImplementedError('the fractal policy body has no gated values / value residual / bias-free or '
                                          'GLU feed-forward / qk norm / xPos rotary / RMSNorm: set attn_gate_values / '
                                          'add_value_residual / ff_no_bias / ff_glu / attn_qk_norm / rotary_xpos / '
                                          'use_rmsnorm to False')
            levels = int(fractal_levels or c.depth)
            self.model = FractalPolicyActorCritic(c, levels).to(dev)
        elif policy_body == 'decoder':
            self.model = WorldModelActorCritic(c).to(dev)
        else:
            raise ValueError(f"policy_body must be 'decoder' or 'fractal', not {policy_body!r}")
        self.policy_body = policy_body
        # the minibatch RSNorm mean (xtrl_minibatch_gather) rides behind the gradient: one all-reduce
        self.flat = FlatParams(self.model, dev, order=self.model.flat_order(), extra=state_dim + 1)
        dist_.broadcast_(self.flat.flat)          # identical initial weights on every rank (DDP semantics)
        if self.gene_pool is not None:
            dist_.broadcast_(self.gene_pool.genes)

        # EMA copy (ema-pytorch semantics restated, xtrl.py:747: EMA(model, beta=ema_decay, **ema_kwargs))
        self.ema_model = copy.deepcopy(self.model)
        for p in self.ema_model.parameters():
            p.grad = None
        self.ema_flat = self.flat.flat.clone()
        self.flat.rebind(self.ema_model, self.ema_flat)
        # split-K weight-gradient partial tiles: one backward's deferred partials (C3 ~190 MB per
        # minibatch) stay resident until its single reduce launch (384 MiB)
        self.gemm_ws = torch.empty(96 << 20, device=dev)
        self.model.bind_flat(self.flat, self.gemm_ws)
        ek = dict(EMA_DEFAULTS)
        unknown = set(ema_kwargs or {}) - set(ek)
        if unknown:
            raise TypeError(f'ema_kwargs {sorted(unknown)} are not supported (known: {sorted(ek)})')
        ek.update(ema_kwargs or {})
        self.ema_beta = ema_decay
        self.ema_update_every, self.ema_update_after = int(ek['update_every']), int(ek['update_after_step'])
        self.ema_inv_gamma, self.ema_power, self.ema_min = float(ek['inv_gamma']), float(ek['power']), \
            float(ek['min_value'])
        self.ema_model_every = ek['update_model_with_ema_every']
        self.ema_model_beta = float(ek['update_model_with_ema_beta'])
        self.ema_step, self.ema_initted = 0, False
        # AdoptAtan2 state over the flat buffer
        n = self.flat.n
        self.opt_m = torch.zeros(n, device=dev)
        self.opt_v = torch.zeros(n, device=dev)
        self.opt_p_init = torch.zeros(n, device=dev) if regen_reg_rate > 0 else None
        self.opt_first = True
        self.opt_cfg = dict(lr=lr, init_lr=lr, betas=tuple(betas), a=1.27, b=1.0, weight_decay=0.,
                            regen_rate=regen_reg_rate, cautious=cautious_factor)
        self.seg_ws = torch.zeros(len(self.flat.params), device=dev, dtype=torch.int32)
        self.opt_chunks = ops.adopt_chunks(self.flat.seg)
        self.norm_ws = torch.zeros(512, device=dev, dtype=torch.float64)
        self.clip_out = torch.zeros(2, device=dev)
        self.max_grad_norm = max_grad_norm
        # RSNorm over [state, reward] (xtrl.py:565-612)
        self.rs_mean = torch.zeros(state_dim + 1, device=dev)
        self.rs_var = torch.ones(state_dim + 1, device=dev)
        self.rs_step = 1
        self.batch_size, self.epochs = batch_size, epochs
        self.lam, self.gamma = lam, gamma
        self.continuous_actions = continuous_actions
        self.save_path = Path(save_path)
        self.actor_loss_weight, self.critic_loss_weight = actor_loss_weight, critic_loss_weight
        self.autoregressive_loss_weight = autoregressive_loss_weight
        self.step = 0
        self.logs = []
        self._deploy = None
        self._genes_dev = None
        self.fused_learn = fused_learn   # False: reference-mode autograd learn step (tests)
        # the world-model heads on the minibatch's valid rows only (XtrlTrainDesc.Tv); False: every row
        self.heads_compact = True
        # host envs: a truncated (not terminated) episode bootstraps GAE from the next state's value
        # (the intent of xtrl.py:1323-1336, whose bootstrap memory lands outside the episode list)
        self.truncation_bootstrap = truncation_bootstrap
        self._train_step = None

    @property
    def device(self):
        return self.accelerator.device

    # ---- checkpoint (xtrl.py:792-806) -----------------------------------------------------------
    def save(self):
        if not self.accelerator.is_main_process:
            return
        torch.save({'model': self.model.state_dict()}, str(self.save_path))

    def load(self):
        if not self.save_path.exists():
            return
        data = torch.load(str(self.save_path), weights_only=True, map_location=self.device)
        with torch.no_grad():
            for k, v in data['model'].items():
                self.model.state_dict()[k].copy_(v)

    # ---- full training state (improves on the reference, which saves the model only) ----------------
    FULL_FORMAT = 'xtrl_amd/2'

    def _by_name(self, flat):
        """A flat-layout buffer as {parameter name: its slice}: a checkpoint independent of the flat
        order, which follows the backward's completion order and changes with the kernels."""
        return {n: flat[a:b].detach().clone() for n, (a, b) in self.flat.index.items()}

    def _from_name(self, flat, saved, what):
        if sorted(saved) != sorted(self.flat.index):
            raise ValueError(f'checkpoint {what}: parameter names differ from this model')
        for n, (a, b) in self.flat.index.items():
            flat[a:b].copy_(saved[n].reshape(-1).to(flat.device))

    def state_dict_full(self):
        """Everything needed to resume bit-for-bit: model (reference key names), the AdoptAtan2
        moments and regen anchor, the EMA weights and schedule, RSNorm statistics, the gene pool,
        the update counter and seed.  Flat-layout buffers are stored per parameter name."""
        out = dict(model=self.model.state_dict(), format=self.FULL_FORMAT,
                   opt_m=self._by_name(self.opt_m), opt_v=self._by_name(self.opt_v),
                   opt_first=torch.tensor(int(self.opt_first)),
                   ema_flat=self._by_name(self.ema_flat), ema_step=torch.tensor(self.ema_step),
                   ema_initted=torch.tensor(int(self.ema_initted)), rs_mean=self.rs_mean, rs_var=self.rs_var,
                   rs_step=torch.tensor(self.rs_step), step=torch.tensor(self.step), seed=torch.tensor(self.seed))
        if self.opt_p_init is not None:
            out['opt_p_init'] = self._by_name(self.opt_p_init)
        if self.gene_pool is not None:
            out.update(genes=self.gene_pool.genes, gene_step=torch.tensor(self.gene_pool.step))
        return out

    def save_checkpoint(self, path=None):
        if not self.accelerator.is_main_process:
            return
        cpu = lambda v: {n: t.detach().cpu() for n, t in v.items()} if isinstance(v, dict) else (   # noqa: E731
            v.detach().cpu() if isinstance(v, torch.Tensor) else v)
        torch.save({k: cpu(v) for k, v in self.state_dict_full().items()}, str(path or self.save_path))

    def load_checkpoint(self, path=None):
        data = torch.load(str(path or self.save_path), weights_only=True, map_location='cpu')
        dev = self.device
        if 'opt_m' in data and data.get('format') != self.FULL_FORMAT:
            # format 1 stored the flat buffers positionally in a flat order that has since changed:
            # pairing them by position would silently give parameters other parameters' moments
            raise ValueError(f"full checkpoint format {data.get('format')!r} stores the optimiser / EMA buffers in "
                             f"an unrecorded flat order; this build reads {self.FULL_FORMAT!r} (per-parameter names)")
        with torch.no_grad():
            for k, v in data['model'].items():
                self.model.state_dict()[k].copy_(v)
            if 'opt_m' not in data:    # a reference-format checkpoint: weights only
                return
            self._from_name(self.opt_m, data['opt_m'], 'opt_m')
            self._from_name(self.opt_v, data['opt_v'], 'opt_v')
            if self.opt_p_init is not None and 'opt_p_init' in data:
                self._from_name(self.opt_p_init, data['opt_p_init'], 'opt_p_init')
            self.opt_first = bool(int(data['opt_first']))
            self._from_name(self.ema_flat, data['ema_flat'], 'ema_flat')
            self.ema_step, self.ema_initted = int(data['ema_step']), bool(int(data['ema_initted']))
            self.rs_mean = data['rs_mean'].to(dev).clone()
            self.rs_var = data['rs_var'].to(dev).clone()
            self.rs_step, self.step, self.seed = int(data['rs_step']), int(data['step']), int(data['seed'])
            if self.gene_pool is not None and 'genes' in data:
                self.gene_pool.genes = data['genes'].clone()
                self.gene_pool.step = int(data['gene_step'])
                self._genes_dev = None
        self._deploy = None

    # ---- genes ------------------------------------------------------------------------------------
    def latent(self, gene_ids):
        return F.normalize(self.genes_device()[gene_ids], dim=-1)

    def genes_device(self):
        if self._genes_dev is None:   # (after an evolve_: an async copy, no mid-learn host wait)
            self._genes_dev = _to_device_async(self.gene_pool.genes.detach(), self.device)
        return self._genes_dev

    # ---- EMA (ema-pytorch update(), restated) ---------------------------------------------------------
    def _ema_update(self):
        step = self.ema_step
        self.ema_step += 1
        should_update = step % self.ema_update_every == 0
        if should_update and step <= self.ema_update_after:
            self.ema_flat.copy_(self.flat.flat)
            return
        if should_update:
            if not self.ema_initted:
                self.ema_flat.copy_(self.flat.flat)
                self.ema_initted = True
            ops.ema_lerp(self.ema_flat, self.flat.flat, 1. - self.ema_decay())
        # ema-pytorch checks update_model_with_ema_every on every step, independent of should_update
        # (parity unpinned: ema-pytorch is not in the container; DESIGN.md decision log)
        if self.ema_model_every is not None and step % self.ema_model_every == 0:
            # the online model takes the EMA weights (ema-pytorch update_model_with_ema)
            ops.ema_lerp(self.flat.flat, self.ema_flat, 1. - self.ema_model_beta)

    def ema_decay(self):
        """ema-pytorch get_current_decay (after the step counter's increment)."""
        epoch = max(self.ema_step - self.ema_update_after - 1, 0)
        if epoch <= 0:
            return 0.
        value = 1 - (1 + epoch / self.ema_inv_gamma) ** -self.ema_power
        return min(max(value, self.ema_min), self.ema_beta)

    # ---- optimiser step: clip_grad_norm_ + AdoptAtan2 + EMA hook (xtrl.py:987-992) ---------------------
    def optimizer_step(self):
        ops.grad_norm(self.flat.grad, self.max_grad_norm, self.norm_ws, self.clip_out)
        o = self.opt_cfg
        ops.adopt_atan2(self.flat.flat, self.flat.grad, self.opt_m, self.opt_v, self.opt_p_init, self.flat.seg,
                        self.opt_chunks, self.seg_ws, self.clip_out, lr=o['lr'], init_lr=o['init_lr'], betas=o['betas'], a=o['a'],
                        b=o['b'], weight_decay=o['weight_decay'], regen_rate=o['regen_rate'], cautious=o['cautious'],
                        first_step=self.opt_first)
        self.opt_first = False
        self._ema_update()

    # ---- learn (xtrl.py:808-1023) -----------------------------------------------------------------
    def learn(self, traj, episode_lens, gene_ids, fitnesses=None, update=None, probe=None, probe_step=None):
        """traj: dict of device tensors [N][Tmax][.] (rollout buffers, padded with zeros).
        ``probe(epoch, minibatch, idx, loss, stats)`` (tests) runs after backward, before the step;
        ``probe_step(epoch, minibatch)`` (tests) right after the optimiser step."""
        c, dev = self.cfg, self.device
        update = self.step if update is None else update
        lens = episode_lens.to(dev, torch.int32)
        N = lens.shape[0]
        lens_host = episode_lens.detach().to('cpu', torch.int64)   # (the learn's one length read)
        n = int(lens_host.max())
        # the genes' fitnesses on the host once per learn (evolve_ reads them on the host after every
        # minibatch: a device tensor there was a host wait per minibatch, the GPU idling while the next
        # minibatch was enqueued)
        if c.evolutionary and fitnesses is not None:
            fitnesses = fitnesses.detach().float().cpu()
        model = self.model
        boot = traj.get('boot')     # host envs: truncation-bootstrap values (NaN: none)
        _, returns = ops.hlgauss_gae(traj['values'], traj['rewards'], traj['bounds'], model.hl_centers, n,
                                     self.gamma, self.lam, boot, lens if boot is not None else None)
        states = traj['states'][:, :n]
        actions = (traj['actions_f'] if c.continuous else traj['actions'])[:, :n]
        rewards = traj['rewards'][:, :n]
        old_lp = traj['logp'][:, :n]
        bounds = traj['bounds'][:, :n]
        old_values = traj['values'][:, :n]
        gene_ids = gene_ids.to(dev)
        rs_mean, rs_var, rs_step = self.rs_mean.clone(), self.rs_var.clone(), self.rs_step
        model.train()
        # the epochs' minibatch orders (host generator: bit parity with torch.randperm), uploaded from
        # pinned memory without a host wait — the learn's only host round trip is the length max above
        perms_host = torch.stack([epoch_permutation(self.seed, update, e, N) for e in range(self.epochs)])
        perms = _to_device_async(perms_host, dev)
        sd = self.rs_var.sqrt().clamp(min=1e-5)
        lo, hi = c.reward_range
        fused = self.fused_learn
        if fused:
            returns = returns.contiguous()
            gather = self.batch_gather(traj['rewards'].shape[1])
        # one stats row per minibatch, written in place by the fused loss (no per-minibatch clone)
        n_mb_epoch = (N + self.batch_size - 1) // self.batch_size
        n_mb = self.epochs * n_mb_epoch
        attn_stride = self.batch_size * c.heads
        assert n_mb * attn_stride < 2 ** 32, "attention dropout counters exceed 32 bits"
        stats_rows = torch.zeros(n_mb, L.LOSS_STATS, device=dev) if fused else None
        logs0 = len(self.logs)
        lat_ep = None
        for epoch in range(self.epochs):
            for mbi, k in enumerate(range(0, N, self.batch_size)):
                idx = perms[epoch, k:k + self.batch_size]
                b = idx.shape[0]
                if fused:   # device minibatch assembly (xtrl_minibatch_gather)
                    g = gather(traj, returns, lens, idx, self.rs_mean, self.rs_var, n)
                    mb_lens, mb_act, prev_act, swr = g['lens'], g['action'], g['prev_action'], g['swr']
                    mb_old_lp, mb_ret, mb_old_v, mb_done = g['old_logp'], g['returns'], g['old_values'], g['dones']
                else:
                    mb_lens = lens[idx].contiguous()
                    mb_act = actions[idx].contiguous()
                    mb_rew = rewards[idx]
                    prev_act = torch.full_like(mb_act, 0. if c.continuous else -1)
                    prev_act[:, 1:] = mb_act[:, :-1]
                    prev_rew = torch.zeros_like(mb_rew)
                    prev_rew[:, 1:] = mb_rew[:, :-1]
                    swr = (torch.cat((states[idx], prev_rew[..., None]), dim=-1) - self.rs_mean) / sd
                    swr = swr.contiguous()
                    mb_old_lp, mb_ret = old_lp[idx].contiguous(), returns[idx].contiguous()
                    mb_old_v, mb_done = old_values[idx].contiguous(), bounds[idx].contiguous()
                keep = reward_coin(self.seed, update, epoch, mbi, c.reward_dropout)
                if c.evolutionary and lat_ep is None:   # per-episode latents, refreshed after an evolve
                    lat_ep = self.latent(gene_ids)
                latent = lat_ep.index_select(0, idx) if c.evolutionary else None
                # dropout streams: every minibatch of the update its own FF counter and a disjoint
                # range of attention counters (layer in the Philox c3 sub-index, include/xtrl_hip.h)
                ordinal = epoch * n_mb_epoch + mbi
                attn_seed, attn_off, ff_off = self.seed * 1000003 + update, ordinal * attn_stride, ordinal
                if self.fused_learn:
                    step = self.train_step(b, n)
                    # the minibatch's valid-token count, from the host copies (no device read)
                    n_valid = int(lens_host[perms_host[epoch, k:k + self.batch_size]].clamp(max=n).sum())
                    step.forward(swr, prev_act, mb_act, latent, mb_lens, keep, attn_seed, attn_off, ff_off,
                                 c.dropout, Tv=n_valid if (self.heads_compact or self.packed_learn) else 0,
                                 packed=self.packed_learn)
                else:
                    act_in = prev_act if c.continuous else prev_act.long()
                    nxt = mb_act if c.continuous else mb_act.long()
                    raw, values, pred_raw, done_logit = model.forward_train(
                        swr[..., :-1], act_in, swr[..., -1], nxt, latent, mb_lens, keep,
                        attn_seed=attn_seed, attn_offset=attn_off, ff_offset=ff_off)
                K = ops.LossConsts(actions=mb_act, old_logp=mb_old_lp, returns=mb_ret, old_values=mb_old_v,
                                   dones=mb_done, lens=mb_lens, real=swr, support=model.hl_support, centers=model.hl_centers,
                                   continuous=c.continuous, squash=c.squash, hl_mean=c.hl_reduction_mean,
                                   eps_clip=c.eps_clip, value_clip=c.value_clip, entropy_weight=c.entropy_weight,
                                   w_actor=self.actor_loss_weight, w_critic=self.critic_loss_weight,
                                   w_autoreg=self.autoregressive_loss_weight, lo=float(lo), hi=float(hi),
                                   sigma=float(model.hl_sigma))
                self.flat.zero_grad()
                if self.fused_learn:
                    stats = step.loss(K, stats_rows[len(self.logs) - logs0])
                    bar = self.bucket_allreduce()
                    step.backward(bar.handles if bar is not None else None)
                    loss = stats[L.LS['loss']]
                    # DDP gradient mean (xtrl.py:981), bucketed and overlapped with the backward; the
                    # RSNorm batch mean (xtrl.py:601) rides in the last bucket's tail
                    if bar is not None:
                        bar.run()
                    else:
                        dist_.mean_(self.flat.grad_ext)
                else:
                    loss, stats = ops.fused_loss(raw, values, pred_raw, done_logit, K)
                    loss.backward()
                    dist_.mean_(self.flat.grad)   # DDP gradient mean (xtrl.py:981)
                if probe is not None:
                    probe(epoch, mbi, idx, loss, stats)
                self.optimizer_step()
                if probe_step is not None:
                    probe_step(epoch, mbi)
                # RSNorm copy update with the normalised masked rows (xtrl.py:1005, 598-610)
                with torch.no_grad():
                    if fused:
                        m = g['rs_m']   # (averaged over ranks with the gradient above)
                        rsnorm_update(rs_mean, rs_var, m, rs_step)
                    else:
                        mask = (torch.arange(n, device=dev)[None, :] < mb_lens[:, None]).float()
                        m = (swr * mask[..., None]).sum((0, 1)) / mask.sum()
                        m = dist_.mean_(m)
                        t = rs_step
                        delta = m - rs_mean
                        rs_mean = rs_mean + delta / t
                        rs_var = (t - 1) / t * (rs_var + delta ** 2 / t)
                    rs_step += 1
                if (c.evolutionary and fitnesses is not None and self.step > self.evolve_after_step
                        and self.step % self.evolve_every == 0):
                    g = torch.Generator().manual_seed(evolve_seed(self.seed, update, epoch, mbi))
                    self.gene_pool.evolve_(fitnesses, generator=g)
                    self._genes_dev = None
                    lat_ep = None
                self.logs.append(stats)
        self.rs_mean, self.rs_var, self.rs_step = rs_mean, rs_var, rs_step
        self.step += 1

    def bucket_allreduce(self):
        """The overlapped bucketed all-reduce of the fused learn step (None: one process, or
        XTRL_DP_BUCKETS=0 for one all-reduce after the backward)."""
        if not dist_.dp_active() or os.environ.get('XTRL_DP_BUCKETS', '1') == '0' \
                or not hasattr(self.model, 'flat_bucket_ranges') or self.flat.flat.device.type != 'cuda':
            return None
        bar = getattr(self, '_bar', None)
        if bar is None:
            self._bar = bar = dist_.BucketAllReduce(self.flat.grad_ext, self.model.flat_bucket_ranges(self.flat))
        return bar

    def batch_gather(self, Tmax):
        bg = getattr(self, '_batch_gather', None)
        if bg is None or bg.n_max < Tmax:
            from .train import BatchGather
            self._batch_gather = bg = BatchGather(self.cfg, self.batch_size, Tmax, self.device, rs_m=self.flat.extra)
        return bg

    def train_step(self, b, n):
        """The fused learn step, with activation buffers for up to (batch_size, n) minibatches."""
        ts = self._train_step
        if ts is None or b > ts.b_max or n > ts.n_max:
            from .train import FractalTrainStep, FusedTrainStep
            cls = FractalTrainStep if self.policy_body == 'fractal' else FusedTrainStep
            self._train_step = ts = cls(self.model, self.flat, self.gemm_ws, max(b, self.batch_size),
                                        max(n, ts.n_max if ts is not None else 0))
        return ts

    def pop_logs(self):
        """Per-minibatch dict(loss, actor_loss, critic_loss, autoreg_loss, pred_done_loss)."""
        if not self.logs:
            return []
        s = torch.stack(self.logs).cpu()
        self.logs = []
        return [dict(loss=float(r[L.LS['loss']]), actor_loss=float(r[L.LS['actor']]),
                     critic_loss=float(r[L.LS['critic']]), autoreg_loss=float(r[L.LS['autoreg']]),
                     pred_done_loss=float(r[L.LS['done']])) for r in s]

    # ---- deploy (xtrl.py:1025-1065): online model, one token per call with a KV cache --------------
    @torch.no_grad()
    def forward(self, state, reward=None, hiddens=None, latent_gene_id=0):
        c = self.cfg
        if self._deploy is None or self._deploy[1] != self.step:
            eng = make_engine(self.model, 1, 4096 if c.dim_head == 16 else 1024, sim_mode=SIM_HOST)
            self._deploy = (eng, self.step)
        eng = self._deploy[0]
        eng.pack(self.model, self.rs_mean, self.rs_var)
        t = 0 if hiddens is None else hiddens['t']
        if hiddens is not None:
            for dst, src in zip(eng.cache_tensors(), hiddens['cache']):
                dst.copy_(src)
        state = torch.as_tensor(np.asarray(state), dtype=torch.float32, device=self.device).reshape(1, -1)
        eng.state.copy_(state)
        latent = self.latent(torch.tensor([latent_gene_id], device=self.device)) if c.evolutionary else None
        eng._begin(self.seed, 0, 0, torch.zeros(1, dtype=torch.int32), latent)
        eng.prev_reward.fill_(0. if reward is None else float(reward))
        eng.desc.no_reward_cond = int(reward is None)
        eng.prev_action.fill_(-1)     # the deploy forward passes no actions (xtrl.py:1056-1061)
        eng.step(t)
        raw = eng.logits[0].clone()
        new_h = dict(t=t + 1, cache=[x.clone() for x in eng.cache_tensors()])
        return raw, new_h


def _to_device_async(t, dev):
    """Host tensor -> device without blocking the host: a pinned staging copy and a non-blocking
    upload (the caching host allocator keeps the pinned block alive until the copy has run)."""
    dev = torch.device(dev)
    if dev.type != 'cuda':
        return t.to(dev)
    return t.contiguous().pin_memory().to(dev, non_blocking=True)


# ----------------------------------------------------------------------------------------------
# Learner (xtrl.py:1069-1380)
# ----------------------------------------------------------------------------------------------


class Learner(nn.Module):
    def __init__(self, state_dim, num_actions, reward_range, world_model: dict, continuous_actions=False,
                 squash_continuous=True, continuous_actions_clamp=None, evolutionary=False, evolve_every=10,
                 evolve_after_step=20, latent_gene_pool: dict | None = None, max_timesteps=500, batch_size=8,
                 num_episodes_per_update=64, lr=0.0008, betas=(0.9, 0.99), lam=0.95, gamma=0.99, eps_clip=0.2,
                 value_clip=0.4, beta_s=.01, regen_reg_rate=1e-4, cautious_factor=0.1, epochs=4, ema_decay=0.9,
                 save_every=100, frac_actor_critic_head_gradient=0.5, accelerate_kwargs: dict = dict(),
                 agent_kwargs: dict = dict(), use_graph=True, shard_by_gene=False):
        super().__init__()
        assert num_episodes_per_update % batch_size == 0   # xtrl.py:1104
        self.accelerator = dist_.DistContext(accelerate_kwargs.get('device') if accelerate_kwargs else None)
        gp = latent_gene_pool if latent_gene_pool is not None else dict(dim=128, num_genes_per_island=3,
                                                                           num_selected=2, tournament_size=2)
        self.agent = Agent(state_dim=state_dim, num_actions=num_actions, continuous_actions=continuous_actions,
                           squash_continuous=squash_continuous, reward_range=reward_range, world_model=world_model,
                           evolutionary=evolutionary, evolve_every=evolve_every, evolve_after_step=evolve_after_step,
                           latent_gene_pool=gp, epochs=epochs, max_timesteps=max_timesteps, batch_size=batch_size,
                           lr=lr, betas=betas, lam=lam, gamma=gamma, beta_s=beta_s, regen_reg_rate=regen_reg_rate,
                           cautious_factor=cautious_factor, eps_clip=eps_clip, value_clip=value_clip,
                           ema_decay=ema_decay, frac_actor_critic_head_gradient=frac_actor_critic_head_gradient,
                           accelerator=self.accelerator, **agent_kwargs)
        self.num_episodes_per_update = num_episodes_per_update
        self.max_timesteps = max_timesteps
        n_genes = self.agent.gene_pool.num_genes if evolutionary else 1
        self.episode_genes = [(e, g) for e in range(num_episodes_per_update) for g in range(n_genes)]
        world, rank = self.accelerator.num_processes, self.accelerator.process_index
        # every rank runs the same number of optimiser steps (one gradient all-reduce each), so the
        # (episode, gene) pairs must split evenly (the reference all-gathers instead, xtrl.py:868-871)
        assert world == 1 or len(self.episode_genes) % world == 0, \
            f'{len(self.episode_genes)} (episode, gene) pairs do not split evenly over {world} processes'
        # shard_by_gene (C5, evolutionary): rank r rolls out every episode of genes g = r (mod world),
        # so with population == world gene g lives on GPU g; otherwise torch.chunk over the pairs
        self.shard_by_gene = bool(shard_by_gene and evolutionary)
        if self.shard_by_gene:
            assert n_genes % world == 0, f'{n_genes} genes do not split evenly over {world} processes'
            mine, slots = dist_.shard_pairs_by_gene(self.episode_genes, world, rank)
            self.episode_genes_for_process, self.slot_offset, self.pair_slots = mine, 0, slots
        else:
            self.episode_genes_for_process, self.slot_offset = dist_.shard_pairs(self.episode_genes, world, rank)
            self.pair_slots = None
        self.num_actions, self.continuous_actions = num_actions, continuous_actions
        self.continuous_actions_clamp = continuous_actions_clamp
        self.save_every = save_every
        self.use_graph = use_graph
        self._engine = None
        self.last_rollout = None

    @property
    def device(self):
        return self.accelerator.device

    # ---- device-sim rollout: all of this rank's (episode, gene) pairs in one batch ----------------
    def _engine_for(self, env, T):
        key = (env.mode, env.hazard_log2, T)
        if self._engine is None or self._engine[0] != key:
            E = len(self.episode_genes_for_process)
            mode = SIM_LANDER if env.mode == 'lander' else SIM_README
            eng = make_engine(self.agent.model, E, T, sim_mode=mode, hazard_log2=env.hazard_log2,
                              clamp=self.continuous_actions_clamp, use_graph=self.use_graph)
            self._engine = (key, eng)
        return self._engine[1]

    def rollout_device(self, env, update, T):
        agent = self.agent
        eng = self._engine_for(env, T)
        eng.pack(agent.ema_model, agent.rs_mean, agent.rs_var)
        pairs = self.episode_genes_for_process
        ep = torch.tensor([e for e, _ in pairs], dtype=torch.int32)
        genes = torch.tensor([g for _, g in pairs], dtype=torch.long, device=self.device)
        latent = agent.latent(genes) if agent.evolutionary else None
        traj = eng.run(agent.seed, update, ep, latent, slot_offset=self.slot_offset, slots=self.pair_slots)
        return traj, eng.lens, genes, eng.cum_reward

    # ---- host-env rollout (xtrl.py:1220-1341) ------------------------------------------------------
    def rollout_host(self, env, update, T, episode_seeds=None):
        """Roll this rank's (episode, gene) pairs out against a host env.  A scalar env (the
        reference contract) runs the pairs one by one exactly like the reference loop; a vectorised
        env (``num_envs`` attribute: ``reset(seed=?) -> states [E][S] | (states, ...)``,
        ``step(actions [E] | [E][A]) -> (states, rewards [E], terminated [E][, truncated [E], ...])``)
        runs the pairs in waves of num_envs, one batched decode step, one action copy to the host
        and one env-result copy to the device per timestep (the env's sub-env i takes the wave's
        i-th pair; sub-envs whose episode ended are still stepped and their results ignored).
        Semantics as the reference: is_boundary = terminated; done = terminated | truncated; a
        4-tuple's 4th item is read as truncated (quirk B8); a truncated, not terminated episode
        bootstraps GAE from the next state's value (xtrl.py:1323-1336; ``truncation_bootstrap``)."""
        agent = self.agent
        c = agent.cfg
        vector = getattr(env, 'num_envs', None) is not None
        W = int(env.num_envs) if vector else 1
        eng = self._engine_for_host(W, T)
        eng.pack(agent.ema_model, agent.rs_mean, agent.rs_var)
        pairs = self.episode_genes_for_process
        N, dev = len(pairs), self.device
        S, A, B = c.state_dim, c.num_actions, c.num_bins
        out = dict(states=torch.zeros(N, T, S, device=dev), actions=torch.zeros(N, T, dtype=torch.int32, device=dev),
                   actions_f=torch.zeros(N, T, A, device=dev) if c.continuous else None,
                   logp=torch.zeros(N, T, A, device=dev) if c.continuous else torch.zeros(N, T, device=dev),
                   rewards=torch.zeros(N, T, device=dev), bounds=torch.zeros(N, T, dtype=torch.uint8, device=dev),
                   values=torch.zeros(N, T, B, device=dev))
        boot = torch.full((N,), float('nan'), device=dev)
        lens = torch.zeros(N, dtype=torch.int32)
        cum = torch.zeros(N, dtype=torch.float64)
        genes = torch.tensor([g for _, g in pairs], dtype=torch.long, device=dev)
        for w0 in range(0, N, W):
            wave = pairs[w0:w0 + W]
            rows = len(wave)
            seeds = None
            if agent.evolutionary and episode_seeds is not None:
                seeds = [int(episode_seeds[e]) for e, _ in wave]
            reset, step = (_vector_env_fns if vector else _scalar_env_fns)(env, W, seeds, c.continuous)
            latent = None
            if agent.evolutionary:   # (the wave's genes sliced on the device: no upload per wave)
                gw = genes[w0:w0 + rows]
                if rows < W:
                    gw = torch.cat((gw, gw.new_zeros(W - rows)))
                latent = agent.latent(gw)
            slots = [self._slot(w0 + i) for i in range(rows)] + [0] * (W - rows)
            traj, wl, wt, wb = eng.run_host_wave(reset, step, agent.seed, update, rows, latent, slots, T,
                                                 bootstrap=agent.truncation_bootstrap)
            keys = [k for k, v in traj.items() if v is not None]
            torch._foreach_copy_([out[k][w0:w0 + rows] for k in keys], [traj[k][:rows, :T] for k in keys])
            lens[w0:w0 + rows] = torch.from_numpy(wl[:rows])
            cum[w0:w0 + rows] = torch.from_numpy(wt[:rows])
            for i in map(int, wb[:rows].nonzero()[0]):
                n = int(wl[i])      # the bootstrap step wrote the next state and its logits at index n
                boot[w0 + i] = agent.model.hl_value(traj['values'][i, n])
                if n < T:
                    out['values'][w0 + i, n].zero_()
                    out['states'][w0 + i, n].zero_()
        out['boot'] = boot
        return out, lens.to(dev), genes, cum

    def _engine_for_host(self, W, T):
        key = ('host', W, T)
        if self._engine is None or self._engine[0] != key:
            eng = make_engine(self.agent.model, W, T + 1, sim_mode=SIM_HOST, clamp=self.continuous_actions_clamp)
            self._engine = (key, eng)
        return self._engine[1]

    def _slot(self, i):
        """Global (episode, gene) pair index of this rank's i-th pair (keys its sampling stream)."""
        return self.pair_slots[i] if self.pair_slots is not None else self.slot_offset + i

    # ---- fitness per gene in pair order (xtrl.py:1345-1346, 1362) -------------------------------------
    def fitness(self, cum_reward, genes):
        agent = self.agent
        if not agent.evolutionary:
            return None
        # the reference's order: per episode a double sum of its rewards (xtrl.py:1282, 1310), then
        # fitnesses[gene] += that sum on an fp32 tensor, episode after episode (xtrl.py:1346) — an fp32
        # add of the fp32-rounded return, sequential per gene in pair order (np.add.at is unbuffered
        # and in index order).  One device->host copy of the episode returns per update; the rank sum
        # (xtrl.py:1362) is the only collective.
        G = agent.gene_pool.num_genes
        cum = cum_reward.detach().to('cpu', torch.float64).numpy().astype(np.float32)
        fit = np.zeros(G, dtype=np.float32)
        np.add.at(fit, genes.detach().cpu().numpy(), cum)
        fit = torch.from_numpy(fit)
        if dist_.is_distributed():
            fit = dist_.sum_(fit.to(self.device)).cpu()
        return fit

    def forward(self, env, num_learning_updates: int, seed=None, max_timesteps=None):
        T = max_timesteps or self.max_timesteps
        agent = self.agent
        if seed is not None:
            torch.manual_seed(seed)
            np.random.seed(seed)
            agent.seed = int(seed)
        device_sim = getattr(env, 'xtrl_device_sim', False)
        for update in range(num_learning_updates):
            u = agent.step
            if device_sim:
                traj, lens, genes, cum = self.rollout_device(env, u, T)
            else:
                seeds = None
                if agent.evolutionary:
                    g = torch.Generator().manual_seed(agent.seed * 31 + u)
                    seeds = torch.randint(0, int(1e7), (self.num_episodes_per_update,), generator=g)
                traj, lens, genes, cum = self.rollout_host(env, u, T, seeds)
            self.last_rollout = (traj, lens, genes)
            self.accelerator.wait_for_everyone()
            fit = self.fitness(cum, genes)
            agent.learn(traj, lens, genes, fit, update=u)
            if update % self.save_every == 0:
                agent.save()
        agent.save()


# ----------------------------------------------------------------------------------------------
# host env contracts (xtrl.py:1232-1305) as batched reset / step closures for run_host_wave
# ----------------------------------------------------------------------------------------------


def _parse_step(o):
    """(next_state, reward, terminated, truncated) of one step return (xtrl.py:1299-1305)."""
    if len(o) >= 4:
        return o[0], o[1], o[2], o[3]
    if len(o) == 3:
        return o[0], o[1], o[2], False
    raise RuntimeError('invalid number of returns from environment .step')


def _scalar_env_fns(env, W, seeds, continuous):
    """The reference's scalar contract: reset(**{seed}) -> state | (state, ...); step(action.tolist())."""
    assert W == 1
    kw = dict(seed=seeds[0]) if seeds is not None else {}

    def reset():
        r = env.reset(**kw)
        return np.asarray(r[0] if isinstance(r, tuple) else r, dtype=np.float32)[None]

    def step(actions, live):
        a = actions[0].tolist() if continuous else int(actions[0])
        ns, r, term, trunc = _parse_step(env.step(a))
        return (np.asarray(ns, dtype=np.float32)[None], np.asarray(r, dtype=np.float64).reshape(-1)[:1],
                np.array([bool(term)]), np.array([bool(trunc)]))

    def step_scalar(a):   # (the gated one-row loop: Python scalars, no per-step arrays)
        return _parse_step(env.step(a))
    step.scalar = step_scalar
    return reset, step


def _vector_env_fns(env, W, seeds, continuous):
    """A vectorised env of W sub-envs: reset(seed=[...]) / step(actions [W] or [W][A])."""
    def flags(x):
        if isinstance(x, dict):
            # a batch-level info dict (gym vector 4-tuple): per-env truncation keys, never bool(dict)
            # — a non-empty infos dict would otherwise truncate every sub-env after one step
            for key in ('TimeLimit.truncated', 'truncated'):
                if key in x:
                    v = np.broadcast_to(np.asarray(x[key]).astype(bool), (W,))
                    has = x.get('_' + key)
                    return v & np.broadcast_to(np.asarray(has).astype(bool), (W,)) if has is not None else v
            return np.zeros(W, dtype=bool)
        if isinstance(x, (list, tuple)) and x and isinstance(x[0], dict):
            return np.array([bool(i) for i in x])
        return np.broadcast_to(np.asarray(x).astype(bool), (W,))

    def reset():
        kw = {}
        if seeds is not None:
            kw = dict(seed=list(seeds) + [0] * (W - len(seeds)))
        r = env.reset(**kw)
        return np.asarray(r[0] if isinstance(r, tuple) else r, dtype=np.float32).reshape(W, -1)

    def step(actions, live):
        ns, r, term, trunc = _parse_step(env.step(actions.copy()))
        return (np.asarray(ns, dtype=np.float32).reshape(W, -1), np.asarray(r, dtype=np.float64).reshape(W),
                flags(term), flags(trunc))
    return reset, step
