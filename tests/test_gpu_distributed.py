"""Two data-parallel ranks on one GPU (gloo carries the collectives; the 8-GPU bench uses RCCL):
both ranks run two full learning updates of the device Learner on their halves of the (episode,
gene) pairs.  After every optimiser step the flat gradient was all-reduced, so the weights, the
EMA copy, the RSNorm statistics and the gene pool must be bitwise identical on the two ranks, and
the rollouts must reproduce a single-process rollout of the same pairs (world-size-invariant
sampling streams)."""
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


def _make(world):
    from xtrl_amd import Learner, SynthVecSim
    torch.manual_seed(3)
    wm = dict(attn_dim_head=16, heads=4, depth=2, attn_gate_values=True, add_value_residual=True,
              learned_value_residual_mix=True)
    learner = Learner(8, 4, (-2., 2.), world_model=wm, max_timesteps=20, batch_size=2, num_episodes_per_update=4,
                      evolutionary=True, evolve_every=1, evolve_after_step=0,
                      latent_gene_pool=dict(dim=8, num_genes_per_island=3, num_selected=2, tournament_size=2),
                      agent_kwargs=dict(dropout=0.1, seed=7, hidden_dim=48, save_path='/tmp/xtrl_dp_test.pt'),
                      use_graph=False)
    return learner, SynthVecSim(8, 4, 'lander', hazard_log2=3)


def _worker(rank, world, port, out_dir):
    sys.path[:0] = [str(REPO), str(REPO / 'x-transformers-rl_amd')]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK='0')
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        learner, env = _make(world)
        traj, lens, _, _ = learner.rollout_device(env, 0, 20)
        first = dict(actions=traj['actions'].cpu().clone(), lens=lens.cpu().clone())
        learner(env, 2)
        a = learner.agent
        torch.save(dict(flat=a.flat.flat.cpu(), ema=a.ema_flat.cpu(), rs_mean=a.rs_mean.cpu(), rs_var=a.rs_var.cpu(),
                        genes=a.gene_pool.genes.clone(), first=first, pairs=learner.episode_genes_for_process),
                   os.path.join(out_dir, f'rank{rank}.pt'))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_two_ranks_one_gpu_stay_in_lockstep(tmp_path):
    world, port = 2, _free_port()
    mp.start_processes(_worker, args=(world, port, str(tmp_path)), nprocs=world, start_method='spawn')
    r = [torch.load(tmp_path / f'rank{i}.pt', weights_only=True) for i in range(world)]
    for k in ('flat', 'ema', 'rs_mean', 'rs_var', 'genes'):
        assert torch.equal(r[0][k], r[1][k]), k
    assert torch.isfinite(r[0]['flat']).all()
    # the concatenated rank rollouts == a single-process rollout of all pairs
    sys.path[:0] = [str(REPO), str(REPO / 'x-transformers-rl_amd')]
    learner, env = _make(1)
    traj, lens, _, _ = learner.rollout_device(env, 0, 20)
    n0 = len(r[0]['pairs'])
    assert torch.equal(torch.cat([r[0]['first']['lens'], r[1]['first']['lens']]), lens.cpu())
    assert torch.equal(torch.cat([r[0]['first']['actions'], r[1]['first']['actions']]), traj['actions'].cpu())
    assert n0 * 2 == lens.numel()
