"""Two data-parallel ranks on one GPU (gloo carries the collectives; the 8-GPU bench uses RCCL).

* lockstep: both ranks run two full learning updates of the device Learner on their halves of
  the (episode, gene) pairs.  After every optimiser step the flat gradient was all-reduced, so the
  weights, the EMA copy, the RSNorm statistics and the gene pool must be bitwise identical on the
  two ranks, and the rollouts must reproduce a single-process rollout of the same pairs
  (world-size-invariant sampling streams).
* DP gradient: the all-reduced gradient of every optimiser step of one update equals the mean of
  the gradients a single process computes on each rank's minibatch separately (the DDP semantics
  of the reference, xtrl.py:885/981: every rank normalises advantages and averages its loss over
  its own minibatch, DDP averages the rank gradients).  The learning rate is 0 so every minibatch
  sees the same weights on both sides; the gradient buffer's tail (the minibatch RSNorm mean,
  xtrl.py:601) is compared too.
* gene-sharded EPO (C5 partition): with ``shard_by_gene`` rank r rolls out every
  episode of genes g = r (mod world); the rank rollouts reassembled in pair order equal the
  single-process rollout, the fitness sums over ranks equal the single-process fitness, and the
  ranks stay in lockstep through evolve_."""
import os
import socket
import sys
from pathlib import Path

import pytest
import torch
import torch.multiprocessing as mp

REPO = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _make(world, shard_by_gene=False, genes=3, episodes=4, fractal=None, evo=True):
    from xtrl_amd import Learner, SynthVecSim
    torch.manual_seed(3)
    wm = dict(attn_dim_head=16, heads=4, depth=2)
    extra = {}
    if fractal:   # the C5 policy body (causal fractal encoder), as bench.py C5 runs it
        extra = dict(policy_body='fractal', fractal_levels=fractal)
    else:
        wm.update(attn_gate_values=True, add_value_residual=True, learned_value_residual_mix=True)
    learner = Learner(8, 4, (-2., 2.), world_model=wm, max_timesteps=20, batch_size=2,
                      num_episodes_per_update=episodes, evolutionary=evo, evolve_every=1, evolve_after_step=0,
                      latent_gene_pool=dict(dim=8, num_genes_per_island=genes, num_selected=2, tournament_size=2),
                      agent_kwargs=dict(dropout=0.1, seed=7, hidden_dim=48, save_path='/tmp/xtrl_dp_test.pt', **extra),
                      use_graph=False, shard_by_gene=shard_by_gene)
    return learner, SynthVecSim(8, 4, 'lander', hazard_log2=3)


def _grad_probe(agent, out):
    def probe(epoch, mbi, idx, loss, stats):
        out.append(agent.flat.grad_ext.detach().cpu().clone())
    return probe


def _worker(rank, world, port, out_dir, mode):
    sys.path[:0] = [str(REPO), str(REPO / 'x-transformers-rl_amd')]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK='0')
    if mode in ('c5grad', 'c5w8'):   # one collective per backward bucket (no coalescing of the small test buckets)
        os.environ['XTRL_DP_BUCKET_FLOATS'] = '1'
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        gene_mode = mode in ('genes', 'c5')
        if mode == 'c5':     # population 8 over 4 ranks (2 genes each), fractal body
            learner, env = _make(world, shard_by_gene=True, genes=8, episodes=2, fractal=2)
        elif mode in ('c5grad', 'c5w8'):   # c5w8: population 8 over 8 ranks, gene g on rank g
            learner, env = _make(world, shard_by_gene=True, genes=8, episodes=2, fractal=2)
        elif mode == 'c4':   # the C4 partition: one policy, the episodes split 8 ways (torch.chunk)
            learner, env = _make(world, episodes=16, evo=False)
        else:
            learner, env = _make(world, shard_by_gene=gene_mode, genes=4 if gene_mode else 3)
        a = learner.agent
        traj, lens, genes, cum = learner.rollout_device(env, 0, 20)
        first = dict(actions=traj['actions'].cpu().clone(), lens=lens.cpu().clone(), fit=learner.fitness(cum, genes))
        grads = []
        from xtrl_amd import distributed as dist_
        coll0 = dist_.COUNTS['all_reduce']
        if mode in ('grad', 'c4', 'c5grad', 'c5w8'):
            lr = a.opt_cfg['lr']
            a.opt_cfg['lr'] = 0.     # weights fixed: every minibatch gradient at the same point
            a.learn(traj, lens, genes, first['fit'], update=0, probe=_grad_probe(a, grads))
            first['allreduces'] = dist_.COUNTS['all_reduce'] - coll0
            first['genes_after'] = a.gene_pool.genes.clone() if a.gene_pool is not None else torch.zeros(1)
            if mode in ('c4', 'c5w8'):   # then one full learning update: the ranks must stay in lockstep
                a.opt_cfg['lr'] = lr
                learner(env, 1)
        else:
            learner(env, 2)
        torch.save(dict(flat=a.flat.flat.cpu(), ema=a.ema_flat.cpu(), rs_mean=a.rs_mean.cpu(), rs_var=a.rs_var.cpu(),
                        genes=a.gene_pool.genes.clone() if a.gene_pool is not None else torch.zeros(1), first=first, pairs=learner.episode_genes_for_process,
                        slots=learner.pair_slots, grads=grads),
                   os.path.join(out_dir, f'rank{rank}.pt'))
    finally:
        dist.destroy_process_group()


def _run(tmp_path, mode, world=2):
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), mode), nprocs=world, start_method='spawn')
    sys.path[:0] = [str(REPO), str(REPO / 'x-transformers-rl_amd')]
    return [torch.load(tmp_path / f'rank{i}.pt', weights_only=True) for i in range(world)]


@pytest.mark.gpu
def test_two_ranks_one_gpu_stay_in_lockstep(tmp_path):
    r = _run(tmp_path, 'lockstep')
    for k in ('flat', 'ema', 'rs_mean', 'rs_var', 'genes'):
        assert torch.equal(r[0][k], r[1][k]), k
    assert torch.isfinite(r[0]['flat']).all()
    # the concatenated rank rollouts == a single-process rollout of all pairs
    learner, env = _make(1)
    traj, lens, _, _ = learner.rollout_device(env, 0, 20)
    n0 = len(r[0]['pairs'])
    assert torch.equal(torch.cat([r[0]['first']['lens'], r[1]['first']['lens']]), lens.cpu())
    assert torch.equal(torch.cat([r[0]['first']['actions'], r[1]['first']['actions']]), traj['actions'].cpu())
    assert n0 * 2 == lens.numel()


@pytest.mark.gpu
def test_dp_gradient_equals_mean_of_rank_minibatch_gradients(tmp_path):
    r = _run(tmp_path, 'grad')
    assert len(r[0]['grads']) == len(r[1]['grads']) > 0
    for g0, g1 in zip(r[0]['grads'], r[1]['grads']):
        assert torch.equal(g0, g1)          # every rank holds the same all-reduced gradient
    # single process: each rank's half of the pairs learned on its own, from the same weights
    learner, env = _make(1)
    a = learner.agent
    a.opt_cfg['lr'] = 0.
    traj, lens, genes, cum = learner.rollout_device(env, 0, 20)
    fit = learner.fitness(cum, genes)
    n0 = len(r[0]['pairs'])
    flat0 = a.flat.flat.clone()
    rs0 = (a.rs_mean.clone(), a.rs_var.clone(), a.rs_step)
    per_rank = []
    for rank in range(2):
        a.rs_mean, a.rs_var, a.rs_step = rs0[0].clone(), rs0[1].clone(), rs0[2]
        a.step = 0
        rows = slice(rank * n0, (rank + 1) * n0)
        sub = {k: (v[rows].contiguous() if v is not None else None) for k, v in traj.items()}
        grads = []
        a.learn(sub, lens[rows].contiguous(), genes[rows].contiguous(), fit, update=0, probe=_grad_probe(a, grads))
        assert torch.equal(a.flat.flat, flat0)     # lr 0: the weights did not move
        per_rank.append(grads)
    steps = len(r[0]['grads'])
    assert len(per_rank[0]) == len(per_rank[1]) == steps
    for i in range(steps):
        want = (per_rank[0][i] + per_rank[1][i]) / 2
        got = r[0]['grads'][i]
        scale = float(want.abs().max())
        err = float((got - want).abs().max())
        assert err <= 1e-6 * scale + 1e-9, (i, err, scale)


@pytest.mark.gpu
def test_gene_sharded_epo_partition(tmp_path):
    r = _run(tmp_path, 'genes')
    # gene g on rank g (mod 2), every episode of the gene
    for rank in range(2):
        assert {g for _, g in r[rank]['pairs']} == {rank, rank + 2}
        assert len(r[rank]['pairs']) == 4 * 2
    for k in ('flat', 'ema', 'rs_mean', 'rs_var', 'genes'):
        assert torch.equal(r[0][k], r[1][k]), k
    # single process, all pairs: the rank rows reassembled by global pair index match
    learner, env = _make(1, genes=4)
    traj, lens, genes, cum = learner.rollout_device(env, 0, 20)
    fit = learner.fitness(cum, genes)
    for rank in range(2):
        slots = torch.tensor(r[rank]['slots'])
        assert torch.equal(r[rank]['first']['lens'], lens.cpu()[slots])
        assert torch.equal(r[rank]['first']['actions'], traj['actions'].cpu()[slots])
        torch.testing.assert_close(r[rank]['first']['fit'], fit, rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
def test_c5_gene_sharded_population8_four_ranks(tmp_path):
    """The C5 partition at world 4: EPO population 8, gene g on rank g (mod 4) — two genes per rank —
    with the fractal policy body, two full learning updates (evolve_ every minibatch).  Ranks stay
    bitwise in lockstep (weights, EMA, RSNorm, genes); each rank's rollout reproduces the single-
    process rollout at its global pair slots and the fitness summed over ranks equals the single-
    process fitness."""
    r = _run(tmp_path, 'c5', world=4)
    for rank in range(4):
        assert {g for _, g in r[rank]['pairs']} == {rank, rank + 4}
        assert len(r[rank]['pairs']) == 2 * 2
    for k in ('flat', 'ema', 'rs_mean', 'rs_var', 'genes'):
        for rank in range(1, 4):
            assert torch.equal(r[0][k], r[rank][k]), (k, rank)
    assert torch.isfinite(r[0]['flat']).all()
    learner, env = _make(1, genes=8, episodes=2, fractal=2)
    traj, lens, genes, cum = learner.rollout_device(env, 0, 20)
    fit = learner.fitness(cum, genes)
    for rank in range(4):
        slots = torch.tensor(r[rank]['slots'])
        assert torch.equal(r[rank]['first']['lens'], lens.cpu()[slots])
        assert torch.equal(r[rank]['first']['actions'], traj['actions'].cpu()[slots])
        torch.testing.assert_close(r[rank]['first']['fit'], fit, rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
def test_c4_eight_ranks_dp_partition(tmp_path):
    """The C4 partition (BASELINE configs[3]: one policy, the episodes sharded 8-way, a gradient
    all-reduce per optimiser step) with 8 ranks on one GPU over gloo, at reduced size (16 episodes,
    2 per rank).  The concatenated rank rollouts equal the single-process rollout; every rank holds
    the same all-reduced gradient at every optimiser step, equal to the mean of the 8 per-rank
    minibatch gradients a single process computes; after a full learning update the 8 ranks'
    weights, EMA and RSNorm statistics are bitwise identical."""
    world = 8
    r = _run(tmp_path, 'c4', world=world)
    learner, env = _make(1, episodes=16, evo=False)
    a = learner.agent
    a.opt_cfg['lr'] = 0.
    traj, lens, genes, cum = learner.rollout_device(env, 0, 20)
    assert torch.equal(torch.cat([r[i]['first']['lens'] for i in range(world)]), lens.cpu())
    assert torch.equal(torch.cat([r[i]['first']['actions'] for i in range(world)]), traj['actions'].cpu())
    n0 = len(r[0]['pairs'])
    assert n0 * world == lens.numel() == 16
    steps = len(r[0]['grads'])
    assert steps > 0
    for i in range(1, world):
        assert len(r[i]['grads']) == steps
        for g0, gi in zip(r[0]['grads'], r[i]['grads']):
            assert torch.equal(g0, gi)
    flat0 = a.flat.flat.clone()
    rs0 = (a.rs_mean.clone(), a.rs_var.clone(), a.rs_step)
    per_rank = []
    for rank in range(world):
        a.rs_mean, a.rs_var, a.rs_step = rs0[0].clone(), rs0[1].clone(), rs0[2]
        a.step = 0
        rows = slice(rank * n0, (rank + 1) * n0)
        sub = {k: (v[rows].contiguous() if v is not None else None) for k, v in traj.items()}
        grads = []
        a.learn(sub, lens[rows].contiguous(), genes[rows].contiguous(), None, update=0, probe=_grad_probe(a, grads))
        assert torch.equal(a.flat.flat, flat0)
        assert len(grads) == steps
        per_rank.append(grads)
    for i in range(steps):
        want = sum(per_rank[k][i] for k in range(world)) / world
        got = r[0]['grads'][i]
        scale = float(want.abs().max())
        assert float((got - want).abs().max()) <= 1e-6 * scale + 1e-9, i
    for k in ('flat', 'ema', 'rs_mean', 'rs_var'):
        for rank in range(1, world):
            assert torch.equal(r[0][k], r[rank][k]), (k, rank)
    assert torch.isfinite(r[0]['flat']).all() and not torch.equal(r[0]['flat'], flat0.cpu())


@pytest.mark.gpu
def test_c5_fractal_bucketed_allreduce_gradient(tmp_path):
    """The fractal learn step's data-parallel gradient at world 4 (C5 partition: population 8, two
    genes per rank): the backward records an event pair per gradient bucket (heads + aggregation, one
    per level, the rest) and the bucket all-reduces overlap it — one collective per bucket per
    optimiser step with coalescing off; every rank holds the same gradient, equal to the mean of the
    four per-rank minibatch gradients a single process computes."""
    world = 4
    r = _run(tmp_path, 'c5grad', world=world)
    steps = len(r[0]['grads'])
    assert steps > 0
    levels = 2
    # per optimiser step: levels + 2 bucket all-reduces (the RSNorm mean rides in the last one)
    assert r[0]['first']['allreduces'] == steps * (levels + 2), (r[0]['first']['allreduces'], steps)
    for i in range(1, world):
        for g0, gi in zip(r[0]['grads'], r[i]['grads']):
            assert torch.equal(g0, gi)
    learner, env = _make(1, genes=8, episodes=2, fractal=2)
    a = learner.agent
    a.opt_cfg['lr'] = 0.
    traj, lens, genes, cum = learner.rollout_device(env, 0, 20)
    fit = learner.fitness(cum, genes)
    flat0 = a.flat.flat.clone()
    rs0 = (a.rs_mean.clone(), a.rs_var.clone(), a.rs_step)
    per_rank = []
    for rank in range(world):
        a.rs_mean, a.rs_var, a.rs_step = rs0[0].clone(), rs0[1].clone(), rs0[2]
        a.step = 0
        rows = torch.tensor(r[rank]['slots'], device=lens.device)
        sub = {k: (v[rows].contiguous() if v is not None else None) for k, v in traj.items()}
        grads = []
        a.learn(sub, lens[rows].contiguous(), genes[rows].contiguous(), fit, update=0, probe=_grad_probe(a, grads))
        assert torch.equal(a.flat.flat, flat0) and len(grads) == steps
        per_rank.append(grads)
    for i in range(steps):
        want = sum(per_rank[k][i] for k in range(world)) / world
        got = r[0]['grads'][i]
        scale = float(want.abs().max())
        assert float((got - want).abs().max()) <= 1e-6 * scale + 1e-9, i


@pytest.mark.gpu
def test_c5_population8_eight_ranks_one_gene_each(tmp_path):
    """The C5 partition exactly as BASELINE configs[4] names it — EPO population 8, ONE gene per rank
    (gene g on rank g), the fractal policy body — with 8 gloo ranks on one GPU at reduced size (2
    episodes per gene).  Each rank's rollout reproduces the single-process rollout at its global pair
    slots and the fitness summed over ranks equals the single-process fitness (x_transformers_rl.py:
    1345-1362); with the learning rate at 0, every optimiser step makes one collective per gradient
    bucket (levels + 2, no coalescing) and every rank holds the same gradient, equal to the mean of the
    8 per-rank minibatch gradients a single process computes; the genes after that update's
    evolve_ calls (evolution.py:76-184, every minibatch) agree with the single process's; after one
    more full learning update the 8 ranks' weights, EMA, RSNorm statistics and genes are bitwise
    identical (x_transformers_rl.py:1143-1154)."""
    world, levels = 8, 2
    r = _run(tmp_path, 'c5w8', world=world)
    for rank in range(world):
        assert {g for _, g in r[rank]['pairs']} == {rank}
        assert len(r[rank]['pairs']) == 2
    steps = len(r[0]['grads'])
    assert steps > 0
    assert r[0]['first']['allreduces'] == steps * (levels + 2), (r[0]['first']['allreduces'], steps)
    for i in range(1, world):
        assert len(r[i]['grads']) == steps
        for g0, gi in zip(r[0]['grads'], r[i]['grads']):
            assert torch.equal(g0, gi)
    learner, env = _make(1, genes=8, episodes=2, fractal=levels)
    a = learner.agent
    a.opt_cfg['lr'] = 0.
    traj, lens, genes, cum = learner.rollout_device(env, 0, 20)
    fit = learner.fitness(cum, genes)
    for rank in range(world):
        slots = torch.tensor(r[rank]['slots'])
        assert torch.equal(r[rank]['first']['lens'], lens.cpu()[slots])
        assert torch.equal(r[rank]['first']['actions'], traj['actions'].cpu()[slots])
        torch.testing.assert_close(r[rank]['first']['fit'], fit, rtol=1e-6, atol=1e-6)
    flat0 = a.flat.flat.clone()
    genes0 = a.gene_pool.genes.clone()
    rs0 = (a.rs_mean.clone(), a.rs_var.clone(), a.rs_step)
    per_rank = []
    for rank in range(world):
        a.rs_mean, a.rs_var, a.rs_step = rs0[0].clone(), rs0[1].clone(), rs0[2]
        a.step = 0
        a.gene_pool.genes.copy_(genes0)
        rows = torch.tensor(r[rank]['slots'], device=lens.device)
        sub = {k: (v[rows].contiguous() if v is not None else None) for k, v in traj.items()}
        grads = []
        a.learn(sub, lens[rows].contiguous(), genes[rows].contiguous(), fit, update=0, probe=_grad_probe(a, grads))
        assert torch.equal(a.flat.flat, flat0) and len(grads) == steps
        per_rank.append(grads)
        # evolve_ sees the same global fitness on every rank: the same genes as the 8-rank run
        torch.testing.assert_close(a.gene_pool.genes.cpu(), r[rank]['first']['genes_after'].cpu(), rtol=0, atol=0)
    for i in range(steps):
        want = sum(per_rank[k][i] for k in range(world)) / world
        got = r[0]['grads'][i]
        scale = float(want.abs().max())
        assert float((got - want).abs().max()) <= 1e-6 * scale + 1e-9, i
    for k in ('flat', 'ema', 'rs_mean', 'rs_var', 'genes'):
        for rank in range(1, world):
            assert torch.equal(r[0][k], r[rank][k]), (k, rank)
    assert torch.isfinite(r[0]['flat']).all() and not torch.equal(r[0]['flat'], flat0.cpu())


def _world1_rccl_worker(rank, port, out_dir):
    """One rank: a learning update's gradients without a process group, then the same update (same
    weights, RSNorm state and minibatches) with a world-1 RCCL group and XTRL_DP_WORLD1=1, so every
    optimiser step's gradient goes through BucketAllReduce: the comm stream waits for the backward's
    per-bucket events and RCCL all-reduces each bucket."""
    sys.path[:0] = [str(REPO), str(REPO / 'x-transformers-rl_amd')]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK='0', WORLD_SIZE='1', LOCAL_RANK='0',
                      XTRL_DP_WORLD1='1', XTRL_DP_BUCKET_FLOATS='1')
    import torch.distributed as dist
    from xtrl_amd import distributed as dist_
    torch.cuda.set_device(0)
    learner, env = _make(1, evo=False)
    a = learner.agent
    a.opt_cfg['lr'] = 0.
    traj, lens, genes, cum = learner.rollout_device(env, 0, 20)
    rs0 = (a.rs_mean.clone(), a.rs_var.clone(), a.rs_step)
    plain = []
    a.learn(traj, lens, genes, None, update=0, probe=_grad_probe(a, plain))
    assert a.bucket_allreduce() is None
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda', 0))
    try:
        a.rs_mean, a.rs_var, a.rs_step = rs0[0].clone(), rs0[1].clone(), rs0[2]
        a.step = 0
        bar = a.bucket_allreduce()
        assert bar is not None and dist.get_backend() == 'nccl'
        rccl = []
        coll0 = dist_.COUNTS['all_reduce']
        a.learn(traj, lens, genes, None, update=0, probe=_grad_probe(a, rccl))
        torch.save(dict(plain=plain, rccl=rccl, allreduces=dist_.COUNTS['all_reduce'] - coll0,
                        buckets=len(bar.groups), depth=a.cfg.depth),
                   os.path.join(out_dir, 'rank0.pt'))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_world1_rccl_bucket_allreduce_leaves_gradient_unchanged(tmp_path):
    """The RCCL data path on hardware: a world-1 ``nccl`` (RCCL) process group forced through
    BucketAllReduce (XTRL_DP_WORLD1=1, one collective per backward bucket).  Every optimiser step's
    gradient — its all-reduce over one rank divided by 1 — equals bitwise the gradient of the same step
    without a process group, and each step makes one RCCL all-reduce per bucket (depth + 2)."""
    mp.start_processes(_world1_rccl_worker, args=(_free_port(), str(tmp_path)), nprocs=1, start_method='spawn')
    r = torch.load(tmp_path / 'rank0.pt', weights_only=True)
    steps = len(r['plain'])
    assert steps > 0 and len(r['rccl']) == steps
    assert r['buckets'] == r['depth'] + 2
    assert r['allreduces'] == steps * r['buckets'], (r['allreduces'], steps, r['buckets'])
    for i, (g0, g1) in enumerate(zip(r['plain'], r['rccl'])):
        assert torch.equal(g0, g1), i


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_self_launches_two_ranks(tmp_path):
    """``python bench.py --gpus 2`` with no launcher starts two ranks itself (torch.distributed.run as a
    child process); under XTRL_BENCH_BACKEND=gloo they share the one GPU.  Rank 0's line reports 2 GPUs,
    the gloo backend, the C3 bucketed all-reduce (3 collectives per optimiser step) and — at N > 1 —
    the PPO loss delta (every rank ran the extra update)."""
    import json
    import subprocess
    env = dict(os.environ, XTRL_BENCH_BACKEND='gloo')
    env.pop('WORLD_SIZE', None)
    p = subprocess.run([sys.executable, '-u', str(REPO / 'bench.py'), '--gpus', '2', '--steps', '1', '--warmup', '0',
                        '--no-cpu-baseline', '--no-roofline'], cwd=str(REPO), env=env, capture_output=True, text=True,
                       timeout=540)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([x for x in p.stdout.splitlines() if x.startswith('{')][-1])
    assert line['n_gpus'] == 2 and line['world_size'] == 2 and line['backend'] == 'gloo'
    assert line['config']['parallelism'] == 'dp2'
    assert line['dp']['world_size'] == 2
    assert line['dp']['grad_allreduces_per_step'] == 3
    assert line['ppo_loss'] is not None and line['ppo_loss']['rel_delta'] <= 1e-4, line['ppo_loss']
