#!/usr/bin/env python
"""Benchmark: env-steps/s of the Learner hot path (rollout + learn) on N MI355X, weak scaling.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c5|c1]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

``--gpus N`` with N > 1 and no launcher around it (no WORLD_SIZE) starts the N ranks itself:
this script re-runs under ``torch.distributed.run`` as a child process (launch_ranks) before the
parent touches the GPU.  Under a launcher, ``--gpus`` must equal WORLD_SIZE.

One "step" = one learning update of the reference Learner loop (xtrl.py:1204-1373): a rollout of
every (episode, gene) pair of this rank on the device Sim, then Agent.learn (GAE + epochs x
minibatches of PPO/world-model updates with clip + AdoptAtan2 + EMA).  Inputs are synthetic
(Philox LunarLander-shaped VecSim) and weights random-init; the timed region contains whole
updates only (no checkpoint writes).

Printed (rank 0, one JSON line): BASELINE metric + roofline of the decode-attention kernel
(HIP events around every launch in the timed region) + the CPU baseline (the oracle's batch-1
restatement of the reference Learner timed on this host) + the PPO loss delta vs that CPU
reference on identical weights and minibatch.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path[:0] = [str(REPO), str(REPO / 'x-transformers-rl_amd')]

import numpy as np   # noqa: E402
import torch         # noqa: E402
import torch.distributed as dist   # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
MFMA_F32_PEAK_TFLOPS = 157.3   # dense fp32 MFMA (v_mfma_f32_32x32x2_f32), MI355X_MICROARCH.md
MFMA_BF16_PEAK_TFLOPS = 16 * MFMA_F32_PEAK_TFLOPS   # dense bf16 MFMA (v_mfma_f32_32x32x16_bf16): 16x the f32 rate
# The large-tile GEMMs compute each fp32 product as six bf16 piece products (csrc/gemm.hip, X6), so
# their MFMA ceiling in fp32-GEMM FLOP/s is the bf16 peak / 6 (XTRL_GEMM_F32=1: native f32 MFMA).
X6_PEAK_TFLOPS = MFMA_BF16_PEAK_TFLOPS / 6

CONFIGS = {
    # configs[2] of BASELINE.json — the north-star workload, per GPU
    'c3': dict(workload='C3: LunarLander-shaped VecSim (S=8, A=4, hazard 1/64), 1024 episodes x 128 steps per '
                        'update per GPU, depth-4 d=256 4x16-head gated value-residual world-model policy, '
                        'batch 128 episodes, 4 epochs, dropout 0.25; no EPO (BASELINE.json configs[2] names no gene pool: one '
                        'policy, actor / critic heads on [embed | state embed], in = 2d)',
               S=8, A=4, episodes=1024, T=128, depth=4, dim=256, heads=4, dim_head=16, gates=True, evo=False,
               batch=128, hazard_log2=6, dropout=0.25, mode='lander'),
    # the C3 model conditioned on an EPO gene pool as train_lander.py runs it (3 genes per island, the
    # heads on [embed | state embed | latent], in = 3d): 384 episodes x 3 genes = 1152 pairs per GPU
    'c3_evo': dict(workload='C3 with EPO (SURVEY 8 C3 "evo: as C2"): LunarLander-shaped VecSim, 384 episodes x 3 '
                            'genes (32-dim) x 128 steps per update per GPU, depth-4 d=256 4x16-head gated '
                            'value-residual policy, heads on [embed | state embed | latent], batch 128, 4 epochs, '
                            'dropout 0.25',
                   S=8, A=4, episodes=384, T=128, depth=4, dim=256, heads=4, dim_head=16, gates=True, evo=True,
                   batch=128, hazard_log2=6, dropout=0.25, mode='lander'),
    # C3 with the per-token critic reduction (hl_reduction_mean=False, decision log) and the packed learn
    # step: the minibatch's valid tokens only (no padding computed; exact for this reduction)
    'c3_tok': dict(workload='C3 with the per-token HL-Gauss critic reduction (hl_reduction_mean=False) and the packed '
                            'learn step (valid tokens only, XtrlTrainDesc.packed): LunarLander-shaped VecSim, 1024 '
                            'episodes x 128 steps per update per GPU, depth-4 d=256 4x16-head gated value-residual '
                            'world-model policy, batch 128 episodes, 4 epochs, dropout 0.25, no EPO',
                   S=8, A=4, episodes=1024, T=128, depth=4, dim=256, heads=4, dim_head=16, gates=True, evo=False,
                   batch=128, hazard_log2=6, dropout=0.25, mode='lander', tok=True),
    # configs[1] — train_lander defaults (evolutionary, 3 genes), 256 episodes, depth-2 d=128
    'c2': dict(workload='C2: LunarLander-shaped VecSim, 256 episodes x 3 genes x 500 steps, depth-2 d=128 EPO',
               S=8, A=4, episodes=256, T=500, depth=2, dim=128, heads=4, dim_head=16, gates=True, evo=True,
               batch=32, hazard_log2=6, dropout=0.25, mode='lander'),
    # C2 with the per-token critic reduction and the packed learn step (85 % of C2's padded token slots
    # are padding: T = 500, mean episode length ~ 64)
    'c2_tok': dict(workload='C2 with the per-token HL-Gauss critic reduction (hl_reduction_mean=False) and the packed '
                            'learn step (valid tokens only): LunarLander-shaped VecSim, 256 episodes x 3 genes x 500 '
                            'steps, depth-2 d=128 EPO',
                   S=8, A=4, episodes=256, T=500, depth=2, dim=128, heads=4, dim_head=16, gates=True, evo=True,
                   batch=32, hazard_log2=6, dropout=0.25, mode='lander', tok=True),
    # configs[4] — EPO population 8, one gene per GPU at 8 GPUs, the fractal policy body (causal per
    # timestep, x-transformers-rl_amd/xtrl_amd/fractal.py); per GPU 1024 (episode, gene) pairs
    'c5': dict(workload='C5 (per GPU): LunarLander-shaped VecSim, EPO population 8 gene-sharded (gene g on GPU g at '
                        '8 GPUs), 1024 episodes x 128 steps per GPU, fractal policy body (4 levels, d=256, 4x16 '
                        'heads, causal per timestep), batch 128 episodes, 4 epochs, dropout 0.25',
               S=8, A=4, episodes=128, genes=8, T=128, depth=4, dim=256, heads=4, dim_head=16, gates=False, evo=True,
               fractal=4, batch=128, hazard_log2=6, dropout=0.25, mode='lander'),
    # the literal drop-in path (train_lander.py:22-70): a scalar host env stepped one action at a time
    # through Learner.rollout_host (the reference's env contract), at train_lander's model shape
    'lander_host': dict(workload='drop-in: train_lander.py shape (EPO 3 genes x 64 episodes, depth 4, d 48, 4x16 heads, '
                                 'batch 8, actor_loss_weight 0.5, frac head gradient 0.1) on a scalar host env '
                                 '(numpy LunarLander-shaped Sim, S=8, A=4, hazard 1/64) through Learner.rollout_host, '
                                 'one env.step per action as the reference loop (xtrl.py:1220-1341)',
                        S=8, A=4, episodes=64, T=500, depth=4, dim=48, heads=4, dim_head=16, gates=True, evo=True,
                        batch=8, hazard_log2=6, dropout=0.25, mode='lander', host=True),
    # the north-star drop-in at its batch (BASELINE.json configs[2] through the host-env path): 1024 numpy
    # LunarLander-shaped sub-envs behind gym's vector-env contract, stepped on the host once per timestep
    # through Learner.rollout_host's vector waves (one batched decode, one action copy to the host and
    # one env-result copy to the device per step), the C3 model
    'lander_hostvec': dict(workload='drop-in at the north-star batch: 1024 numpy LunarLander-shaped host sub-envs '
                                    '(vector-env contract, S=8, A=4, hazard 1/64) x 128 steps through '
                                    'Learner.rollout_host vector waves, C3 model (depth 4, d=256, 4x16-head gated '
                                    'value-residual), batch 128 episodes, 4 epochs, dropout 0.25, no EPO',
                           S=8, A=4, episodes=1024, T=128, depth=4, dim=256, heads=4, dim_head=16, gates=True,
                           evo=False, batch=128, hazard_log2=6, dropout=0.25, mode='lander', host=True, vector=1024),
    # configs[0] — README Sim plumbing case
    'c1': dict(workload='C1: README Sim (S=5, A=2, T=10), depth 1, d=48, 64 episodes, batch 8',
               S=5, A=2, episodes=64, T=10, depth=1, dim=48, heads=4, dim_head=16, gates=False, evo=False,
               batch=8, hazard_log2=0, dropout=0.25, mode='readme'),
}


class HostLanderSim:
    """A scalar host env with the reference's contract (reset(seed=?) -> (state, info); step(action) ->
    (state, reward, terminated, truncated, info), train_lander.py's gym interface): LunarLander-shaped
    (S = 8 N(0, 1) states, A = 4 actions, action-dependent N(0, 1) rewards, termination hazard
    2^-hazard_log2), numpy on the host — one Python call per env step, as gym's LunarLander."""

    def __init__(self, S, A, hazard_log2, seed=0):
        self.S, self.A, self.p = S, A, 2.0 ** -hazard_log2
        self.rng = np.random.default_rng(seed)

    def reset(self, seed=None):
        if seed is not None:
            self.rng = np.random.default_rng(int(seed))
        return self.rng.standard_normal(self.S).astype(np.float32), {}

    def step(self, action):
        state = self.rng.standard_normal(self.S).astype(np.float32)
        reward = float(self.rng.standard_normal() + 0.1 * (int(action) - self.A / 2))
        return state, reward, bool(self.rng.random() < self.p), False, {}


class HostLanderVec:
    """W LunarLander-shaped sub-envs behind gym's vector-env contract (num_envs; reset(seed=[...]) ->
    (states [W][S], info); step(actions [W]) -> (states, rewards [W], terminated [W], truncated [W],
    info)), the same distributions as HostLanderSim, drawn for all sub-envs at once by numpy on the
    host (gym's SyncVectorEnv steps its LunarLanders one by one; the host cost here is the numpy draw)."""

    def __init__(self, W, S, A, hazard_log2, seed=0):
        self.num_envs, self.S, self.A, self.p = W, S, A, 2.0 ** -hazard_log2
        self.rng = np.random.default_rng(seed)

    def reset(self, seed=None):
        if seed is not None:
            self.rng = np.random.default_rng([int(x) for x in np.asarray(seed).reshape(-1)[:4]])
        return self.rng.standard_normal((self.num_envs, self.S), dtype=np.float32), {}

    def step(self, actions):
        W = self.num_envs
        state = self.rng.standard_normal((W, self.S), dtype=np.float32)
        reward = self.rng.standard_normal(W) + 0.1 * (np.asarray(actions).reshape(W) - self.A / 2)
        term = self.rng.random(W) < self.p
        return state, reward, term, np.zeros(W, dtype=bool), {}


def build_learner(cfg, seed, use_graph=True, world=1):
    from xtrl_amd import Learner, SynthVecSim
    wm = dict(attn_dim_head=cfg['dim_head'], heads=cfg['heads'], depth=cfg['depth'])
    if cfg['gates']:
        wm.update(attn_gate_values=True, add_value_residual=True, learned_value_residual_mix=True)
    extra = dict(policy_body='fractal', fractal_levels=cfg['fractal']) if cfg.get('fractal') else {}
    if cfg.get('host') and not cfg.get('vector'):   # train_lander.py:42-49
        extra.update(actor_loss_weight=0.5)
    if cfg.get('tok'):
        extra.update(hl_reduction_mean=False, packed_learn=True)
    learner = Learner(state_dim=cfg['S'], num_actions=cfg['A'], reward_range=(-5., 5.), world_model=wm,
                      max_timesteps=cfg['T'], batch_size=cfg['batch'],
                      num_episodes_per_update=cfg['episodes'] * world,   # weak scaling: episodes per GPU fixed
                      evolutionary=cfg['evo'], evolve_every=5, evolve_after_step=10,
                      latent_gene_pool=dict(dim=32, num_genes_per_island=cfg.get('genes', 3), num_selected=2,
                                            tournament_size=2),
                      agent_kwargs=dict(hidden_dim=cfg['dim'], dropout=cfg['dropout'], seed=seed,
                                        save_path='/tmp/xtrl_bench_ppo.pt', **extra),
                      use_graph=use_graph, shard_by_gene=bool(cfg.get('fractal')),
                      **(dict(frac_actor_critic_head_gradient=0.1) if cfg.get('host') and not cfg.get('vector') else {}))
    # (C5: episodes per update = 128 x world over 8 genes, gene-sharded: 1024 pairs per GPU at any N)
    if cfg.get('vector'):
        return learner, HostLanderVec(cfg['vector'], cfg['S'], cfg['A'], cfg['hazard_log2'], seed)
    if cfg.get('host'):
        return learner, HostLanderSim(cfg['S'], cfg['A'], cfg['hazard_log2'], seed)
    env = SynthVecSim(cfg['S'], cfg['A'], cfg['mode'], cfg['hazard_log2'])
    return learner, env


PHASES = []   # (start, after rollout, after learn) events of the timed updates
HOST_TIMES = {}   # host envs: seconds of the timed updates' steps in decode (+ wait) / env step / feedback


def one_update(learner, env, T, probe=None, phases=False):
    agent = learner.agent
    u = agent.step
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)] if phases else None
    if ev:
        ev[0].record()
    if isinstance(env, (HostLanderSim, HostLanderVec)):   # host envs (Learner.forward's host branch)
        g = torch.Generator().manual_seed(agent.seed * 31 + u)
        seeds = torch.randint(0, int(1e7), (learner.num_episodes_per_update,), generator=g) if agent.evolutionary else None
        traj, lens, genes, cum = learner.rollout_host(env, u, T, seeds)
        if phases:   # the host side of the timed updates' steps (rollout.run_host_wave)
            for k, v in learner._engine[1].host_times.items():
                HOST_TIMES[k] = HOST_TIMES.get(k, 0) + v
    else:
        traj, lens, genes, cum = learner.rollout_device(env, u, T)
    if ev:
        ev[1].record()
    fit = learner.fitness(cum, genes)
    steps = lens.sum()
    agent.learn(traj, lens, genes, fit, update=u, probe=probe)
    if ev:
        ev[2].record()
        PHASES.append(ev)
    agent.logs = []
    return steps, lens


class DecodeAttnTimer:
    """HIP events around every attention-decode launch of the timed region (XtrlDecodeDesc.prof_events),
    on the rollout stream."""

    def __init__(self, learner, env, T):
        import ctypes as C
        eng = learner._engine_for(env, T)
        self.eng, self.L, self.T = eng, eng.c.depth, T
        self.events = [torch.cuda.Event(enable_timing=True) for _ in range(2 * T * self.L)]
        for e in self.events:     # torch creates the HIP event lazily, on first record
            e.record()
        self.arr = (C.c_void_p * len(self.events))(*[e.cuda_event for e in self.events])
        eng.desc.prof_events = C.cast(self.arr, C.POINTER(C.c_void_p))
        eng.graph = None          # re-capture with the event records inside
        self.ms, self.launches, self.bytes = 0.0, 0, 0.0

    def collect(self, lens):
        """After an update: add kernel time and algorithmic bytes of its T*L launches."""
        torch.cuda.synchronize()
        lens = lens.cpu().numpy()
        # the steps with a live episode (the rollout stops launching sub-graphs once none is live,
        # so the event pairs of later steps may not belong to this update), and decoded by the
        # multi-kernel step (the row-resident step of a long tail has no separate attention launch)
        T_eff = min(int(lens.max()), getattr(self.eng, 'rows_from_step', self.T))
        for i in range(T_eff * self.L):
            self.ms += self.events[2 * i].elapsed_time(self.events[2 * i + 1])
        self.launches += T_eff * self.L
        c = self.eng.c
        H, dh = c.heads, c.dim_head
        if T_eff == 0:
            return
        t = np.arange(T_eff)
        alive = (lens[None, :] > t[:, None]).sum(1)                  # live episodes at step t
        # per live (env, head): read K,V rows 0..t-1 (2 t dh f32) + its q|k|v(|gate|mix) row
        # (3 dh, + dh + 1 with gates / mix) (+ the value-residual row dh); write K,V at t (2 dh) +
        # output (dh)
        row = 3 * dh + (dh if c.gate_values else 0) + (1 if c.learned_mix else 0)
        vres = dh if c.value_residual else 0
        per_head = 4.0 * (2 * t * dh + row + vres + 2 * dh + dh)
        self.bytes += float(self.L * (alive * H * per_head).sum())

    def detach(self):
        self.eng.desc.prof_events = None
        self.eng.graph = None


class WgradGemmTimer:
    """HIP events around every launch of the dominant learn kernel — the 128x128-tile
    weight-gradient GEMM k_gemm<2,2,1,2,2,T,T,...> — inside xtrl_train_backward (XtrlTrainDesc
    prof_events / prof_flops), on the learn stream, over the timed region."""

    # the 128x128 weight-gradient launches: the warp-specialised kernel when the split grid is one
    # resident round (the C3 shapes), the register-staged one otherwise
    KERNELS = ('k_gemm_ws<true, true', 'k_gemm<2, 2, 1, 2, 2, true, true')

    def __init__(self, agent, T, cap=8192):
        import ctypes as C
        self.C, self.cap, self.T = C, cap, T
        self.events = [torch.cuda.Event(enable_timing=True) for _ in range(2 * cap)]
        for e in self.events:
            e.record()
        torch.cuda.synchronize()
        self.arr = (C.c_void_p * (2 * cap))(*[e.cuda_event for e in self.events])
        self.flops = (C.c_double * cap)()
        self.n = C.c_int(0)
        self.agent = agent
        self.ms, self.launches, self.total_flops = 0.0, 0, 0.0

    def attach(self):
        # buffers sized for the longest episode (a later, longer update would otherwise rebuild
        # the train step and drop the event pointers)
        D = self.agent.train_step(self.agent.batch_size, self.T).D
        D.prof_events = self.C.cast(self.arr, self.C.POINTER(self.C.c_void_p))
        D.prof_flops = self.C.cast(self.flops, self.C.c_void_p)
        D.prof_cap = self.cap
        D.prof_n = self.C.cast(self.C.pointer(self.n), self.C.c_void_p)
        self.n.value = 0

    def collect(self):
        torch.cuda.synchronize()
        if self.n.value >= self.cap:
            raise RuntimeError(f'WgradGemmTimer: {self.cap} event pairs filled, launches went unrecorded')
        for i in range(self.n.value):
            self.ms += self.events[2 * i].elapsed_time(self.events[2 * i + 1])
            self.total_flops += self.flops[i]
        self.launches += self.n.value
        self.n.value = 0

    def detach(self):
        D = self.agent._train_step.D
        D.prof_events, D.prof_flops, D.prof_cap, D.prof_n = None, None, 0, None


def _profile(kind, config):
    """Newest committed profile of ``kind`` for a bench config: profiles/rNN_<kind>.<ext> for the
    default C3 line, profiles/rNN_<kind>_<config>.<ext> for the others (tools/gpu_check.sh)."""
    import glob
    suffix = '' if config == 'c3' else f'_{config}'
    ext = 'json' if kind == 'pmc_traffic' else 'csv'
    files = sorted(glob.glob(str(Path(__file__).resolve().parent / 'profiles' / f'r[0-9][0-9]_{kind}{suffix}.{ext}')))
    return files[-1] if files else None


def pmc_traffic(config, *kernels):
    """HBM bytes per launch of the kernels whose names contain one of ``kernels`` (dispatch-weighted
    mean) from the newest committed PMC summary of this config (profiles/rNN_pmc_traffic[_cfg].json,
    written by tools/gpu_check.sh pmc from rocprofv3 --pmc passes of this bench: 2 x FETCH_SIZE +
    WRITE_SIZE, the gfx950 correction of the MI355X guide)."""
    path = _profile('pmc_traffic', config)
    if path is None:
        return None
    data = json.load(open(path))
    hits = [v for k, v in data.items() if any(x in k for x in kernels)]
    n = sum(h['dispatches'] for h in hits)
    return round(sum(h['traffic'] * h['dispatches'] for h in hits) / n) if n else None


def rocprof_avg_us(config, *kernels):
    """Average duration (us, call-weighted) of the kernels whose names contain one of ``kernels``
    in the newest committed `rocprofv3 --kernel-trace --stats` summary of this config's bench
    (profiles/rNN_kernel_stats[_cfg].csv) — the profiler's clock beside the bench's HIP events."""
    import csv
    path = _profile('kernel_stats', config)
    if path is None:
        return None
    calls = total = 0
    with open(path) as f:
        for row in csv.DictReader(f):
            if any(k in row['Name'] for k in kernels):
                calls += int(row['Calls'])
                total += float(row['TotalDurationNs'])
    return round(total / calls / 1e3, 2) if calls else None


def pmc_mfma_busy(config, *kernels):
    """Matrix-core busy fraction of the kernels (dispatch-weighted mean of SQ_VALU_MFMA_BUSY_CYCLES /
    (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs), the third PMC pass of tools/gpu_check.sh pmc), or None."""
    path = _profile('pmc_traffic', config)
    if path is None:
        return None
    data = json.load(open(path))
    hits = [v for k, v in data.items() if any(x in k for x in kernels) and 'mfma_busy' in v]
    n = sum(h['dispatches'] for h in hits)
    return round(sum(h['mfma_busy'] * h['dispatches'] for h in hits) / n, 4) if n else None


def algorithmic_work(c, levels, lens, epochs):
    """SURVEY 8(d) algorithmic work per executed env-step of the model ``c`` (ModelConfig; ``levels``:
    the fractal body's level count, None = the decoder): rollout FLOPs, update FLOPs (3 x epochs x
    (rollout + world-model heads)) and decode K/V bytes, with t_bar = the mean number of keys a step
    attends over (its position + 1) across the executed steps of ``lens``."""
    lens = np.asarray(lens, dtype=np.float64)
    t_bar = float((lens * (lens + 1) / 2).sum() / max(lens.sum(), 1))
    d, S, A, B, H = c.dim, c.state_dim, c.num_actions, c.num_bins, c.heads
    I, ff = c.heads * c.dim_head, c.dim * c.ff_mult
    n_out = A * (2 if c.continuous else 1)
    in_dim = d * (3 if c.evolutionary else 2)
    heads = 2 * in_dim * 2 * d * 2 + 2 * 2 * d * (n_out + B) + (2 * c.dim_gene * d if c.evolutionary else 0)
    embed = 4 * S * d
    if levels is None:
        L = c.depth
        n_qkv = 3 * I + (I if c.gate_values else 0)
        body = L * (2 * d * n_qkv + 2 * I * d + 2 * 2 * d * ff + 4 * I * t_bar)
        body += (L - 1) * 2 * d * H if (c.value_residual and c.learned_mix) else 0
    else:
        L = levels
        body = L * (2 * d * 3 * I + 2 * I * d + 2 * 2 * d * I + 2 * 2 * d * ff + 2 * 2 * d * d + 4 * I * t_bar)
        body += 2 * (L + 1) * d * 2 * d + 2 * 2 * d * d
    rollout = body + embed + heads
    update = 3 * epochs * (rollout + 4 * d * d + 4 * d * (S + 1) + 4 * d)
    kv = L * 2 * t_bar * I * 4 + L * 2 * I * 4
    return dict(rollout_flops=rollout, update_flops=update, kv_bytes=kv, t_bar=t_bar)


def total_roofline(value, work, mfma_busy):
    """env-steps/s against the SURVEY 8(d) total roof: per env-step max(rollout FLOPs / peak, K/V
    bytes / HBM) + update FLOPs / peak, at the fp32 MFMA peak SURVEY prices it on and at the
    split-bf16 (X6) peak the GEMMs run at."""
    def roof(peak_tf):
        t = max(work['rollout_flops'] / (peak_tf * 1e12), work['kv_bytes'] / (HBM_PEAK_GBS * 1e9)) + \
            work['update_flops'] / (peak_tf * 1e12)
        return 1.0 / t
    r32, r6 = roof(MFMA_F32_PEAK_TFLOPS), roof(X6_PEAK_TFLOPS)
    return dict(achieved=round(value, 1), unit='env-steps/s', roof=round(r32), frac=round(value / r32, 4),
                peak='fp32 MFMA %.1f TF/s (SURVEY 8(d)), HBM %.0f GB/s' % (MFMA_F32_PEAK_TFLOPS, HBM_PEAK_GBS),
                roof_x6=round(r6), frac_x6=round(value / r6, 4),
                peak_x6='split-bf16 (X6) %.1f TF/s = bf16 dense peak / 6' % X6_PEAK_TFLOPS,
                rollout_mflop_per_step=round(work['rollout_flops'] / 1e6, 3),
                update_mflop_per_step=round(work['update_flops'] / 1e6, 3),
                kv_kb_per_step=round(work['kv_bytes'] / 1e3, 1), t_bar=round(work['t_bar'], 2),
                mfma_busy_dominant_kernel=mfma_busy)


def host_cores():
    """Physical cores of this host (psutil), and the CPU share this process may use (affinity)."""
    try:
        import psutil
        phys = psutil.cpu_count(logical=False)
    except Exception:
        phys = None
    try:
        share = len(os.sched_getaffinity(0))
    except Exception:
        share = os.cpu_count()
    return phys, share


def cpu_baseline(cfg, seed, budget_s, threads=None, episodes=None, reps=5):
    """The oracle's batch-1 CPU restatement of the reference Learner (rollout + learn): ``reps``
    updates (seeds seed .. seed + reps - 1) on a bounded number of episodes of the same workload,
    the median rate reported (BASELINE.md's plan: the median of >= 5 updates)."""
    from oracle import ref_port as R
    threads = threads or int(os.environ.get('OMP_NUM_THREADS', '0')) or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    episodes = episodes or (32 if cfg.get('fractal') else 96 if cfg['T'] >= 100 else 512)
    per = max(2, episodes // reps)   # episodes per update: the whole sample split over the reps
    batch = min(8, per)
    factory = None
    if cfg.get('fractal'):
        from oracle import fractal_ref as FR
        factory = lambda mc: FR.OracleFractalPolicy(mc, cfg['fractal'])   # noqa: E731
    rates, steps_all, t_roll, t_learn = [], 0, 0., 0.
    for r in range(reps):
        c = R.LearnerConfig(cfg['S'], cfg['A'], (-5., 5.), dim=cfg['dim'], depth=cfg['depth'], heads=cfg['heads'],
                            dim_head=cfg['dim_head'], gate_values=cfg['gates'], value_residual=cfg['gates'],
                            learned_mix=cfg['gates'], evolutionary=False, max_timesteps=cfg['T'], batch_size=batch,
                            num_episodes_per_update=per, sim_mode=cfg['mode'], hazard_log2=cfg['hazard_log2'],
                            seed=seed + r, dropout=cfg['dropout'])
        oracle = R.OracleLearner(c, model_factory=factory)
        t0 = time.perf_counter()
        eps, fit = oracle.rollout(0)
        t1 = time.perf_counter()
        oracle.learn(eps, fit, 0)
        t2 = time.perf_counter()
        steps = sum(ep['len'] for ep in eps)
        rates.append(steps / (t2 - t0))
        steps_all, t_roll, t_learn = steps_all + steps, t_roll + (t1 - t0), t_learn + (t2 - t1)
    return dict(value=float(np.median(rates)), unit='env-steps/s', cores=threads, kind='port',
                rates=[round(x, 1) for x in rates],
                sample=f'median of {reps} updates x {per} episodes ({steps_all} env-steps in all), batch {batch}, '
                       f'same model/config, rollout {t_roll:.1f}s + learn {t_learn:.1f}s in all '
                       f'(oracle/ref_port.OracleLearner, batch-1 KV-cached decode like xtrl.py:1250-1341)')


def ppo_loss_delta(learner, env, cfg, check=True):
    """|L_gpu - L_cpu| / |L_cpu| on the first minibatch of one more update, identical weights /
    RSNorm / minibatch tensors; the CPU side is the oracle's restatement.  Every rank
    runs the update (its learn all-reduces gradients); ``check`` (rank 0) compares its local first
    minibatch, the others return None."""
    from oracle import ref_port as R
    from oracle import thirdparty as tp
    agent = learner.agent
    c = agent.cfg
    out = {}
    tp.HLGaussLoss.default_reduction = 'mean' if c.hl_reduction_mean else 'none'   # the agent's reduction
    saved_p = c.dropout
    c.dropout = 0.          # dropout masks are not shared with the CPU side
    u = agent.step
    traj, lens, genes, cum = learner.rollout_device(env, u, cfg['T'])
    mc = R.ModelConfig(c.state_dim, c.num_actions, c.dim, c.depth, c.heads, c.dim_head, cfg['T'], c.reward_range,
                       c.num_bins, c.continuous, c.squash, c.evolutionary, c.dim_gene, c.frac_head_grad,
                       c.entropy_weight, c.eps_clip, c.value_clip, 0., c.reward_dropout, True, c.gate_values,
                       c.value_residual, c.learned_mix)
    if cfg.get('fractal'):
        from oracle import fractal_ref as FR
        model = FR.OracleFractalPolicy(mc, cfg['fractal'])
    else:
        model = R.OracleWMAC(mc)

    def probe(epoch, mbi, idx, loss, stats):
        if out or not check:
            return
        try:   # (never raise out of the learn loop: at N > 1 the other ranks are inside its collectives)
            compare(epoch, mbi, idx, loss)
        except Exception as e:
            out['error'] = repr(e)

    def compare(epoch, mbi, idx, loss):
        idx_c = idx.cpu()
        n = int(lens.max())
        sel = lambda t: t[idx_c][:, :n].cpu()
        states, actions = sel(traj['states']), sel(traj['actions']).long()
        rewards, old_lp, bounds = sel(traj['rewards']), sel(traj['logp']), sel(traj['bounds']).bool()
        values = sel(traj['values'])
        mb_lens = lens.cpu()[idx_c].long()
        hl = model.hl
        full_v = traj['values'][:, :n].cpu()
        returns = R.calc_gae(traj['rewards'][:, :n].cpu(), hl(full_v), (~traj['bounds'][:, :n].cpu().bool()).float(),
                             agent.gamma, agent.lam)[idx_c]
        model.load_state_dict({k: v.detach().cpu() for k, v in agent.model.state_dict().items()})
        model.train()
        rs = R.RSNormState(c.state_dim + 1)
        rs.mean, rs.var = agent.rs_mean.cpu().clone(), agent.rs_var.cpu().clone()
        mb = R.Minibatch(states, actions, rewards, old_lp, returns, values, bounds, genes.cpu()[idx_c], mb_lens)
        from xtrl_amd.learner import reward_coin
        keep = reward_coin(agent.seed, u, epoch, mbi, c.reward_dropout)
        latent = R.l2norm(agent.gene_pool.genes[mb.gene_ids]) if c.evolutionary else None
        ref, _, _, _ = R.minibatch_loss(model, rs, mb, latent, R.LossWeights(agent.actor_loss_weight,
                                                                            agent.critic_loss_weight,
                                                                            agent.autoregressive_loss_weight), keep)
        out.update(gpu=float(loss.detach()), cpu=float(ref.detach()))

    agent.learn(traj, lens, genes, learner.fitness(cum, genes), update=u, probe=probe)
    agent.logs = []
    c.dropout = saved_p
    if not check:
        return None
    if 'error' in out:
        return dict(error=out['error'])
    out['rel_delta'] = abs(out['gpu'] - out['cpu']) / max(abs(out['cpu']), 1e-12)
    return out


def launch_ranks(n):
    """``python bench.py --gpus N`` (N > 1) outside a launcher: run this script under
    ``torch.distributed.run`` with N local ranks (one per GPU, or ranks sharing the GPUs under
    XTRL_BENCH_BACKEND=gloo) as a CHILD process and return its exit code — the parent never
    initialises the GPU (device_count() only reads the topology), so nothing is exec-ed over a live
    HIP context.  Rank 0's line is the job's line."""
    import socket
    import subprocess
    backend = os.environ.get('XTRL_BENCH_BACKEND', 'nccl')
    have = torch.cuda.device_count()
    if backend == 'nccl' and have < n:
        print(f'bench.py: --gpus {n} needs {n} GPUs, {have} visible (XTRL_BENCH_BACKEND=gloo shares them)',
              file=sys.stderr)
        return 2
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')   # RCCL over dmabuf IPC (the pool's driver)
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
           '--master-addr', '127.0.0.1', '--master-port', str(port), str(Path(__file__).resolve()), *sys.argv[1:]]
    print(f'[bench] launching {n} ranks: {" ".join(cmd[1:])}', file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--config', default='c3', choices=sorted(CONFIGS))
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-graph', action='store_true')
    ap.add_argument('--no-roofline', action='store_true')
    ap.add_argument('--no-loss-delta', action='store_true')
    args = ap.parse_args()

    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        # no launcher: start the N ranks ourselves (before this process touches the GPU)
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        raise SystemExit(f'bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks')
    if world > 1:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        # XTRL_BENCH_BACKEND=gloo: multi-rank rehearsal on fewer GPUs than ranks (ranks share devices)
        backend = os.environ.get('XTRL_BENCH_BACKEND', 'nccl')
        dev = local if backend == 'nccl' else local % torch.cuda.device_count()
        torch.cuda.set_device(dev)
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', dev))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    cfg = CONFIGS[args.config]
    torch.manual_seed(args.seed)
    learner, env = build_learner(cfg, args.seed, use_graph=not args.no_graph, world=world)
    T = cfg['T']

    def progress(msg):   # stderr progress outside the timed region (long multi-rank runs stay visibly alive)
        print(f'[bench rank {rank}] {msg}', file=sys.stderr, flush=True)

    for i in range(args.warmup):
        one_update(learner, env, T)
        progress(f'warmup update {i + 1}/{args.warmup}')
    host = bool(cfg.get('host'))
    # Roofline timers — HIP events around every decode-attention launch (inside the captured rollout
    # graph) and every weight-gradient GEMM launch of the learn step — run in a PROBED pass of
    # untimed updates before the headline region (value_probed: its rate), then come out again; the
    # headline region below carries no probe events.
    timer = gtimer = None
    value_probed = None
    if not args.no_roofline and not host:
        timer = DecodeAttnTimer(learner, env, T)
        # capture the rollout graph with the event records inside, and count the weight-gradient
        # launches of one update to size the probed pass's event pool exactly
        probe_timer = WgradGemmTimer(learner.agent, T, cap=1 << 14)
        probe_timer.attach()
        one_update(learner, env, T)
        per_update = probe_timer.n.value
        probe_timer.detach()
        timer.ms, timer.launches, timer.bytes = 0.0, 0, 0.0
        n_probed = max(1, min(args.steps, 3))
        gtimer = WgradGemmTimer(learner.agent, T, cap=per_update * n_probed + 64)
        gtimer.attach()
        torch.cuda.synchronize()
        tp0 = time.perf_counter()
        probed_steps = torch.zeros((), device='cuda', dtype=torch.int64)
        for _ in range(n_probed):
            steps, lens_p = one_update(learner, env, T)
            probed_steps += steps
        torch.cuda.synchronize()
        value_probed = float(probed_steps) / (time.perf_counter() - tp0)
        timer.collect(lens_p)          # the event pairs hold the last probed update's T*L launches
        gtimer.collect()
        gtimer.detach()
        timer.detach()
        progress(f'probed pass: {n_probed} updates, {value_probed:.0f} env-steps/s')
        one_update(learner, env, T)    # re-capture the rollout graph without the event records
    if world > 1:
        dist.barrier()
    from xtrl_amd import distributed as dist_
    coll0 = dict(dist_.COUNTS)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    total = torch.zeros((), device='cuda', dtype=torch.int64)
    lens_last = None
    per_update = []
    for _ in range(args.steps):
        steps, lens = one_update(learner, env, T, phases=True)
        total += steps
        per_update.append(steps)
        lens_last = lens
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    progress(f'timed: {args.steps} updates in {elapsed:.2f} s')
    lens_last = lens_last.cpu().numpy() if lens_last is not None else None
    el = torch.tensor([elapsed], device='cuda', dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(total)
    elapsed = float(el)
    env_steps = int(total)
    # the median per-update rate beside the mean: each timed update's env-steps over its
    # event-timed duration (rollout start -> learn end on the stream; the host gap between updates is
    # not in it), summed / max-ed over ranks like the headline
    upd_steps = torch.stack(per_update).to(torch.float64)
    upd_ms = torch.tensor([e[0].elapsed_time(e[2]) for e in PHASES[-args.steps:]], device='cuda', dtype=torch.float64)
    if world > 1:
        dist.all_reduce(upd_steps)
        dist.all_reduce(upd_ms, op=dist.ReduceOp.MAX)
    upd_rate = (upd_steps / upd_ms * 1e3).cpu()
    value_median = float(upd_rate.median())
    ms_median = float(upd_ms.cpu().median())
    # collectives of the timed updates (per rank): the bucketed gradient all-reduces, RSNorm rides in
    # the last bucket, fitness sums
    coll = {k: (dist_.COUNTS[k] - coll0[k]) / args.steps for k in coll0} if world > 1 else None
    value = env_steps / elapsed

    # committed profiles of this config's bench (profiles/rNN_*[_cfg])
    prof = lambda f, *k: f(args.config, *k)   # noqa: E731

    phase_ms = dict(rollout=round(sum(e[0].elapsed_time(e[1]) for e in PHASES) / len(PHASES), 2),
                    learn=round(sum(e[1].elapsed_time(e[2]) for e in PHASES) / len(PHASES), 2))
    roofline = attn_roofline = None
    if gtimer is not None and gtimer.launches:
        avg_s = gtimer.ms / gtimer.launches / 1e3
        flops = gtimer.total_flops / gtimer.launches
        achieved = flops / avg_s / 1e12
        x6 = os.environ.get('XTRL_GEMM_F32', '0') in ('', '0')
        peak = X6_PEAK_TFLOPS if x6 else MFMA_F32_PEAK_TFLOPS
        roofline = dict(kernel='k_gemm_ws<T,T> / k_gemm<2,2,1,2,2,T,T> (learn-step weight-gradient GEMM, '
                               '128x128 tiles, split-K over 192 workgroups, on the backward side stream beside '
                               'the input-gradient chain; the largest kernel of the update; fp32 products as ' +
                               ('six bf16 piece products, peak = bf16 dense peak / 6)' if x6 else
                                'native f32 MFMA)'), bound='mfma', achieved=round(achieved, 2),
                        peak=round(peak, 1), unit='TFLOP/s', frac=round(achieved / peak, 4),
                        traffic=prof(pmc_traffic, *WgradGemmTimer.KERNELS),
                        mfma_busy=prof(pmc_mfma_busy, *WgradGemmTimer.KERNELS), avg_launch_us=round(avg_s * 1e6, 2),
                        avg_launch_us_rocprof=prof(rocprof_avg_us, *WgradGemmTimer.KERNELS),
                        flops_per_launch=round(flops), launches=gtimer.launches,
                        timed_in='probed pass (events around each launch), not the headline region')
    if timer is not None and timer.launches:
        avg_s = timer.ms / timer.launches / 1e3
        achieved = timer.bytes / timer.launches / avg_s / 1e9
        tail = ('the fused out-projection and both post-norm add + LayerNorms of its rows (fractal body)'
                if cfg.get('fractal') else 'the fused out-projection + residual + FF1 LayerNorm of its rows')
        attn_roofline = dict(kernel=f'k_attn_decode (rollout decode attention over the KV cache, with {tail})', bound='hbm',
                             achieved=round(achieved, 1), peak=HBM_PEAK_GBS, unit='GB/s',
                             frac=round(achieved / HBM_PEAK_GBS, 4), traffic=prof(pmc_traffic, 'k_attn_decode'),
                             avg_launch_us=round(avg_s * 1e6, 2), bytes_per_launch=round(timer.bytes / timer.launches))
        # the profiler's per-launch time (no event records around the launch) and the fraction it gives
        us = prof(rocprof_avg_us, 'k_attn_decode')
        if us:
            attn_roofline.update(avg_launch_us_rocprof=us, frac_rocprof=round(
                timer.bytes / timer.launches / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4))

    total_roof = None
    if lens_last is not None:
        ag = learner.agent
        work = algorithmic_work(ag.cfg, cfg.get('fractal'), lens_last, ag.epochs)
        total_roof = total_roofline(value, work, roofline.get('mfma_busy') if roofline else None)
    loss_delta = None
    cpu = None
    # the loss-delta check runs one more update on EVERY rank (its learn all-reduces gradients; rank 0
    # compares its local first minibatch with the CPU restatement), then the process group ends and
    # rank 0 alone times the CPU baseline, so no rank waits in a collective the others never enter
    if not (args.no_loss_delta or host):
        try:
            loss_delta = ppo_loss_delta(learner, env, cfg, check=(rank == 0))
        except Exception as e:   # reported, never hidden
            loss_delta = dict(error=repr(e))
    backend_name = dist.get_backend() if world > 1 else None
    coll_dp = None
    if coll is not None:
        mb = learner.agent.epochs * (len(learner.episode_genes_for_process) // learner.agent.batch_size)
        coll_dp = dict(backend=backend_name, world_size=dist.get_world_size(), collectives_per_update=coll,
                       optimiser_steps_per_update=mb, grad_allreduces_per_step=round(coll['all_reduce'] / mb, 3))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, args.seed, 20.)
        phys, share = host_cores()
        one = cpu_baseline(cfg, args.seed, 20., threads=1,
                           episodes=8 if cfg.get('fractal') else 32 if cfg['T'] >= 100 else 128, reps=3)
        cpu.update(host_physical_cores=phys, host_cpu_share=share,
                   single_thread=dict(value=one['value'], cores=1, sample=one['sample']))
    if rank == 0:
        line = dict(metric='env-steps/s (rollout+update)', value=round(value, 1), unit='env-steps/s', n_gpus=world,
                    value_median=round(value_median, 1), ms_per_step_median=round(ms_median, 2),
                    value_probed=None if value_probed is None else round(value_probed, 1),
                    steps=args.steps, warmup=args.warmup, ms_per_step=round(1e3 * elapsed / args.steps, 2),
                    higher_is_better=True, scaling='weak', vs_baseline=None, dtype='f32',
                    backend=backend_name or 'single-process', world_size=world,
                    data=('synthetic (numpy LunarLander-shaped host vector env, random-init weights)' if cfg.get('vector') else
                          'synthetic (numpy LunarLander-shaped scalar host env, random-init weights)' if host else
                          'synthetic (Philox LunarLander-shaped VecSim on device, random-init weights)'),
                    config=dict(workload=cfg['workload'],
                                global_batch=cfg['episodes'] * (cfg.get('genes', 3) if cfg['evo'] else 1) * world,
                                seq_len=T, parallelism=f'dp{world}', env_steps=env_steps),
                    roofline=roofline, attention_roofline=attn_roofline, total_roofline=total_roof,
                    cpu_baseline=cpu, ppo_loss=loss_delta,
                    phase_ms=phase_ms)
        if HOST_TIMES.get('steps'):
            n = HOST_TIMES['steps']
            line['host_step_us'] = dict(
                {k: round(1e6 * HOST_TIMES[k] / n, 1) for k in ('decode', 'env', 'feedback')}, steps=n,
                note='per host-env step, host clock: decode = the decode launches + the wait for the actions '
                     '(device->host copy included); env = the env step; feedback = staging + host->device copy + '
                     'the feedback kernel launch')
        if coll_dp is not None:
            line['dp'] = coll_dp
        print(json.dumps(line), flush=True)


if __name__ == '__main__':
    main()
