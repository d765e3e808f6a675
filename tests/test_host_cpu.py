"""CPU-only checks of the product's host side and of the C-ABI library (no kernel launches)."""
import ctypes
import os
import sys
import re
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import philox as OP
from oracle import ref_port as R

REPO = Path(__file__).resolve().parent.parent


def test_library_exports_every_declared_symbol():
    from xtrl_amd import _lib
    lib = _lib.load()
    header = (REPO / 'include' / 'xtrl_hip.h').read_text()
    declared = set(re.findall(r'^\s*(?:int|int64_t|float|const char\*)\s+(xtrl_\w+)\s*\(', header, re.M))
    assert len(declared) >= 18
    for name in declared:
        assert hasattr(lib, name), name
    assert set(_lib.SIGNATURES) <= declared | {'xtrl_last_error'}
    assert lib.xtrl_abi_version() == _lib.ABI_VERSION


@pytest.mark.parametrize('T,b,d,A', [(64 * 500, 64, 128, 1), (16384, 128, 256, 4), (10, 2, 48, 2), (17, 1, 8, 16)])
def test_train_partial_workspace_covers_every_reduction(T, b, d, A):
    """xtrl_train_part_floats (host-only) states the partial-sum floats a learn step needs: the
    LayerNorm backward's 16-row blocks (ceil(T / 16) d), the column sums (min(1024, T / 16) d), the
    latent gradient (b d) and one embedding chunk (A d) — the Python side sizes from it, so a
    1-action env at 64 x 500 tokens (beyond the old (T / 64 + 1) d sizing) fits."""
    from xtrl_amd import _lib
    need = _lib.load().xtrl_train_part_floats(T, b, d, A)
    assert need >= -(-T // 16) * d
    assert need >= min(1024, max(1, T // 16)) * d and need >= b * d and need >= A * d


def test_struct_layouts_match_header():
    """ctypes mirrors of the C structs: field order / count as declared in include/xtrl_hip.h."""
    from xtrl_amd import _lib
    header = (REPO / 'include' / 'xtrl_hip.h').read_text()
    for cname, py in (('XtrlDecodeLayer', _lib.DecodeLayer), ('XtrlDecodeDesc', _lib.DecodeDesc),
                      ('XtrlLossDesc', _lib.LossDesc), ('XtrlRngState', _lib.RngState),
                      ('XtrlTrainLayer', _lib.TrainLayer), ('XtrlTrainDesc', _lib.TrainDesc)):
        body = re.search(r'typedef struct %s \{(.*?)\} %s;' % (cname, cname), header, re.S).group(1)
        body = re.sub(r'/\*.*?\*/', '', body, flags=re.S)
        names = []
        for decl in body.split(';'):
            decl = decl.strip()
            if not decl:
                continue
            decl = re.sub(r'^(const\s+)?\w+\s*\**', '', decl)   # drop the type of the first declarator
            for part in decl.split(','):
                part = part.strip().lstrip('*').strip()
                part = re.sub(r'^(const\s+)?(int|float|uint8_t|int32_t|int64_t|uint32_t|uint64_t|double|XtrlDecodeLayer|XtrlRngState|XtrlTrainLayer)\s*\**\s*', '', part)
                if part:
                    names.append(part)
        assert names == [f[0] for f in py._fields_], (cname, names, [f[0] for f in py._fields_])


@pytest.mark.parametrize('args', [(0, 0, 0, 0, 4, 0), (7, 3, 11, 5, 1, 2), (2 ** 40 + 5, 9, 1000, 499, 2, 0)])
def test_host_rng_matches_oracle_philox(args):
    from xtrl_amd import _lib
    seed, upd, slot, t, field, sub = args
    lib = _lib.load()
    u = lib.xtrl_rng_uniform(seed, upd, slot, t, field, sub)
    z = lib.xtrl_rng_normal(seed, upd, slot, t, field, sub)
    assert np.float32(u) == OP.philox_uniform(seed, upd, slot, t, field, sub + 1)[sub]
    assert np.float32(z) == OP.philox_uniform(seed, upd, slot, t, field, sub + 1, normal=True)[sub]


def test_minibatch_order_and_reward_coin_match_oracle():
    from xtrl_amd.learner import epoch_permutation, reward_coin
    for args in ((0, 0, 0, 10), (5, 3, 2, 129), (123, 7, 3, 1024)):
        assert torch.equal(epoch_permutation(*args), OP.epoch_permutation(*args))
    for seed in range(5):
        for mb in range(6):
            for p in (0., 0.25, 0.5):
                assert reward_coin(seed, 1, 2, mb, p) == OP.reward_coin(seed, 1, 2, mb, p)


def test_shard_pairs_is_torch_chunk():
    from xtrl_amd.distributed import shard_pairs
    for n, world in ((64, 1), (64, 8), (30, 4), (3, 3), (10, 3)):
        pairs = torch.cartesian_prod(torch.arange(n), torch.arange(1))
        chunks = pairs.chunk(world, dim=0)
        for rank in range(world):
            mine, start = shard_pairs([tuple(p) for p in pairs.tolist()], world, rank)
            ref = chunks[rank].tolist() if rank < len(chunks) else []
            assert [list(p) for p in mine] == ref
            if mine:
                assert [list(p) for p in [tuple(x) for x in pairs.tolist()][start:start + len(mine)]] == ref


def test_gene_pool_matches_reference_golden(golden):
    """Product LatentGenePool.evolve_ vs the reference's evolve_ (golden, same generator seeds)."""
    from xtrl_amd.evolution import LatentGenePool
    g = golden('evolve')
    for case in range(3):
        islands, per, sel, tourn, steps = (int(x) for x in g[f'c{case}_cfg'])
        pool = LatentGenePool(dim=8, num_genes_per_island=per, num_selected=sel, tournament_size=tourn,
                              num_islands=islands, migrate_genes_every=10)
        pool.genes = torch.from_numpy(g[f'c{case}_genes0'])
        for s in range(steps):
            gen = torch.Generator().manual_seed(1000 + 10 * case + s)
            selected = pool.evolve_(torch.from_numpy(g[f'c{case}_fitnesses'][s]), generator=gen)
            np.testing.assert_allclose(pool.genes.numpy(), g[f'c{case}_genes'][s], rtol=1e-6, atol=1e-6)
            np.testing.assert_array_equal(selected.numpy(), g[f'c{case}_selected'][s])


@pytest.mark.parametrize('evo,gates,cont', [(False, False, False), (True, True, False), (False, True, True)])
def test_state_dict_layout_matches_reference_names(evo, gates, cont):
    from xtrl_amd.model import ModelConfig, WorldModelActorCritic
    mc = ModelConfig(5, 3, 32, depth=2, evolutionary=evo, dim_gene=8 if evo else 0, continuous=cont,
                     gate_values=gates, value_residual=gates, learned_mix=gates)
    ours = WorldModelActorCritic(mc).state_dict()
    rc = R.ModelConfig(5, 3, 32, depth=2, evolutionary=evo, dim_gene=8 if evo else 0, continuous=cont,
                       gate_values=gates, value_residual=gates, learned_mix=gates)
    ref = R.OracleWMAC(rc).state_dict()
    assert list(ours.keys()) == list(ref.keys())
    for k in ours:
        assert ours[k].shape == ref[k].shape, k


def test_model_state_dict_loads_golden_reference_weights(golden):
    """The reference's own WorldModelActorCritic state_dict (golden) loads into the product model."""
    from xtrl_amd.model import ModelConfig, WorldModelActorCritic
    g = golden('model_forward')
    mc = ModelConfig(6, 4, 32, depth=2, evolutionary=True, dim_gene=8, gate_values=True, value_residual=True,
                     learned_mix=True, reward_range=(-2., 2.))
    m = WorldModelActorCritic(mc)
    sd = {k[3:]: torch.from_numpy(g[k]) for k in g.files if k.startswith('sd.')}
    m.load_state_dict(sd, strict=True)


def test_flat_params_views():
    from xtrl_amd.model import ModelConfig, WorldModelActorCritic
    from xtrl_amd.params import FlatParams
    m = WorldModelActorCritic(ModelConfig(5, 2, 16, depth=1))
    before = {k: v.clone() for k, v in m.state_dict().items()}
    fp = FlatParams(m, 'cpu')
    for k, v in m.state_dict().items():
        assert torch.equal(v, before[k])
    fp.flat.add_(1.)
    assert torch.equal(m.reward_embed, before['reward_embed'] + 1)
    (m.reward_embed.sum() * 2).backward()
    assert torch.equal(fp.grad[:m.reward_embed.numel()], torch.full_like(m.reward_embed, 2.))


def test_flat_layout_aligns_gemm_weights():
    """Every GEMM weight of the C3 model starts 16-byte aligned in the flat buffer (float4 operand
    loads in the HIP GEMM), and the concatenated operands stay adjacent."""
    from xtrl_amd.model import ModelConfig, WorldModelActorCritic
    from xtrl_amd.params import FlatParams
    c = ModelConfig(8, 4, dim=256, depth=4, heads=4, dim_head=16, gate_values=True, value_residual=True,
                    learned_mix=True, evolutionary=True, dim_gene=32)
    m = WorldModelActorCritic(c)
    flat = FlatParams(m, 'cpu', order=m.flat_order())
    for name, (a, b) in flat.index.items():
        p = dict(m.named_parameters())[name]
        if p.dim() == 2 and p.shape[1] % 4 == 0:
            assert a % 4 == 0, (name, a)
    flat.span(['to_pred.0.weight', 'to_pred_done.0.weight'])
    flat.span(['action_head.0.weight', 'critic_head.0.weight'])


def test_full_checkpoint_roundtrip(tmp_path):
    """save_checkpoint / load_checkpoint restore the whole training state (model with reference
    key names, optimiser moments, EMA, RSNorm, gene pool, counters); a reference-format
    {'model': state_dict} file still loads as weights only."""
    from xtrl_amd import Learner
    torch.manual_seed(0)
    kw = dict(world_model=dict(attn_dim_head=16, heads=4, depth=1), evolutionary=True,
              latent_gene_pool=dict(dim=8, num_genes_per_island=3, num_selected=2, tournament_size=2),
              num_episodes_per_update=4, batch_size=2, accelerate_kwargs=dict(device='cpu'),
              agent_kwargs=dict(hidden_dim=16, save_path=str(tmp_path / 'ppo.pt')), use_graph=False)
    a = Learner(5, 2, (-1., 1.), **kw).agent
    with torch.no_grad():
        a.flat.flat.normal_()
        a.opt_m.normal_()
        a.opt_v.uniform_()
        a.ema_flat.normal_()
        a.rs_mean.normal_()
        a.rs_var.uniform_()
        a.gene_pool.genes.normal_()
    a.opt_first, a.ema_step, a.ema_initted, a.rs_step, a.step, a.gene_pool.step = False, 37, True, 9, 4, 2
    a.save_checkpoint()
    torch.manual_seed(1)
    b = Learner(5, 2, (-1., 1.), **kw).agent
    b.load_checkpoint()
    for x, y in ((a.flat.flat, b.flat.flat), (a.opt_m, b.opt_m), (a.opt_v, b.opt_v), (a.ema_flat, b.ema_flat),
                 (a.rs_mean, b.rs_mean), (a.rs_var, b.rs_var), (a.gene_pool.genes, b.gene_pool.genes)):
        assert torch.equal(x, y)
    assert (b.opt_first, b.ema_step, b.ema_initted, b.rs_step, b.step, b.gene_pool.step) == (False, 37, True, 9, 4, 2)
    # the flat-layout buffers are stored per parameter name, so a build whose flat order differs
    # restores every parameter's own moments / EMA weights
    data = torch.load(str(tmp_path / 'ppo.pt'), weights_only=True)
    assert data['format'] == 'xtrl_amd/2' and sorted(data['opt_m']) == sorted(a.flat.index)
    name0 = a.flat.names[0]
    lo, hi = a.flat.index[name0]
    assert torch.equal(data['opt_m'][name0].reshape(-1), a.opt_m[lo:hi])
    # a format-1 file (positional flat buffers, order unrecorded) is refused, not mis-paired
    data.update(format='xtrl_amd/1', opt_m=a.opt_m.clone())
    torch.save(data, str(tmp_path / 'v1.pt'))
    with pytest.raises(ValueError, match='flat order'):
        b.load_checkpoint(tmp_path / 'v1.pt')
    # reference format: weights only (xtrl.py:792-806)
    a.save()
    c = Learner(5, 2, (-1., 1.), **kw).agent
    c.load_checkpoint()
    assert torch.equal(c.flat.flat, a.flat.flat) and c.step == 0


def test_vector_env_info_dict_is_read_per_env():
    """A gym-style vector 4-tuple (obs, rew, done, infos) carries ONE batch-level dict: truncation is
    read from its per-env keys ('TimeLimit.truncated' with the '_TimeLimit.truncated' presence
    mask), never as bool(dict) — which would truncate every sub-env whenever infos is non-empty."""
    from xtrl_amd.learner import _vector_env_fns
    W = 4

    class VecEnv:
        num_envs = W

        def __init__(self, info):
            self.info = info

        def reset(self, seed=None):
            return np.zeros((W, 3))

        def step(self, actions):
            return np.zeros((W, 3)), np.ones(W), np.array([False, True, False, False]), self.info

    cases = [({'episode': {'r': np.zeros(W)}}, [False] * 4),
             ({'TimeLimit.truncated': np.array([True, False, True, False]),
               '_TimeLimit.truncated': np.array([True, True, False, False])}, [True, False, False, False]),
             ({'TimeLimit.truncated': np.array([False, False, False, True])}, [False, False, False, True]),
             ([{}, {'x': 1}, {}, {}], [False, True, False, False])]
    for info, want in cases:
        _, step = _vector_env_fns(VecEnv(info), W, None, False)
        ns, r, term, trunc = step(np.zeros(W, dtype=np.int32), np.ones(W, dtype=bool))
        assert trunc.tolist() == want, (info, trunc)
        assert term.tolist() == [False, True, False, False]


def test_world_model_option_validation():
    """x-transformers Decoder kwargs: implementation switches (attn_flash) are accepted, options the
    MI355X decoder does not implement are refused loudly (xtrl.py:721-734 splats world_model)."""
    from xtrl_amd import Learner
    kw = dict(num_episodes_per_update=2, batch_size=2, accelerate_kwargs=dict(device='cpu'),
              agent_kwargs=dict(hidden_dim=16), use_graph=False)
    a = Learner(5, 2, (-1., 1.), world_model=dict(attn_dim_head=16, heads=4, depth=1, attn_flash=True), **kw).agent
    assert a.cfg.depth == 1 and a.cfg.heads == 4
    with pytest.raises(NotImplementedError):
        Learner(5, 2, (-1., 1.), world_model=dict(attn_dim_head=16, heads=4, depth=1, ff_swish=True), **kw)


def test_world_model_options_defaults_accepted_others_named():
    """world_model options at their x-transformers default build the same network (accepted); the
    implementation switches attn_flash / attn_onnxable are accepted; ff_no_bias builds bias-free
    feed-forward Linears, ff_glu the GLU project-in (x-transformers GLU: ff.0.proj [2 ff][d] with a
    bias); an option the MI355X decoder does not implement raises, naming it."""
    from xtrl_amd import Learner
    kw = dict(num_episodes_per_update=2, batch_size=2, accelerate_kwargs=dict(device='cpu'),
              agent_kwargs=dict(hidden_dim=16), use_graph=False)
    base = dict(attn_dim_head=16, heads=4, depth=1)
    a = Learner(5, 2, (-1., 1.), world_model=dict(base, attn_flash=True, ff_glu=False, attn_qk_norm=False,
                                                  rotary_xpos=False, pre_norm=True, ff_no_bias=False), **kw)
    b = Learner(5, 2, (-1., 1.), world_model=dict(base), **kw)
    assert list(a.agent.model.state_dict()) == list(b.agent.model.state_dict())
    c = Learner(5, 2, (-1., 1.), world_model=dict(base, ff_no_bias=True), **kw)
    names = list(c.agent.model.state_dict())
    assert not any(n.endswith(('ff.0.0.bias', 'ff.2.bias')) for n in names)
    assert len(names) == len(list(b.agent.model.state_dict())) - 2
    g = Learner(5, 2, (-1., 1.), world_model=dict(base, ff_glu=True), **kw).agent.model.state_dict()
    proj = [k for k in g if k.endswith('ff.0.proj.weight')]
    assert len(proj) == 1 and tuple(g[proj[0]].shape) == (2 * 4 * 16, 16)
    assert tuple(g[proj[0].replace('weight', 'bias')].shape) == (2 * 4 * 16,)
    assert not any(k.endswith('ff.0.0.weight') for k in g)
    for opt in (dict(ff_swish=True), dict(macaron=True), dict(use_scalenorm=True), dict(attn_kv_heads=2)):
        with pytest.raises(NotImplementedError, match=next(iter(opt))):
            Learner(5, 2, (-1., 1.), world_model=dict(base, **opt), **kw)
    with pytest.raises(AssertionError, match='causality'):   # x-transformers Decoder refuses the flag
        Learner(5, 2, (-1., 1.), world_model=dict(base, causal=True), **kw)
    # attn_qk_norm / rotary_xpos build the same parameters (the qk norm has no dim scale, the xPos
    # table is not a parameter)
    q = Learner(5, 2, (-1., 1.), world_model=dict(base, attn_qk_norm=True, rotary_xpos=True), **kw)
    assert list(q.agent.model.state_dict()) == list(b.agent.model.state_dict())
    assert q.agent.cfg.qk_norm and q.agent.cfg.rotary_xpos and q.agent.cfg.qk_norm_scale == 10.
    # use_rmsnorm: x-transformers RMSNorm's gain is named g (LayerNorm's gamma)
    r = Learner(5, 2, (-1., 1.), world_model=dict(base, use_rmsnorm=True), **kw).agent.model.state_dict()
    assert [k.replace('.gamma', '.g') for k in b.agent.model.state_dict()] == list(r)


def test_bench_refuses_gpus_world_size_mismatch():
    """Under a launcher, ``--gpus`` must equal WORLD_SIZE (bench.py exits before touching the GPU)."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE='2', RANK='0', LOCAL_RANK='0')
    p = subprocess.run([sys.executable, str(REPO / 'bench.py'), '--gpus', '1'], env=env, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode != 0 and 'WORLD_SIZE=2' in p.stderr
