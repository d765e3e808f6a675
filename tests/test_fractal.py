"""Fractal policy body: parameter-layout KATs on CPU, HIP forward vs the oracle on GPU.

Pins: the parameter counts printed by the reference's comprehensive_demo.py (:338-357) for its three
architectures, and the parameter names / shapes of the committed checkpoint
fractal_experiments/frala_easy_final/final_fractal_agent.pt (tests/golden/fractal_easy_layout.json,
made by tests/golden/make_fractal_layout.py).  The forward numerics of the reference's own fractal
arithmetic (level embedding, post-norm block order, global-state update, level projections, final
aggregation, heads) are pinned by tests/test_fractal_golden.py: oracle/fractal_ref.py reproduces the
reference's fractal_rl.py run in the build container (tests/golden/fractal.npz) to fp32 rounding.
Only the x-transformers Attention / FeedForward internals inside those modules remain the
restatement's (x-transformers is absent).  The GPU tests compare the HIP path with that oracle, in
fp64, within 1e-4 of the output scale."""
import json
import math
from pathlib import Path

import pytest
import torch

from oracle import fractal_ref as FR

REPO = Path(__file__).resolve().parent.parent
GOLDEN = REPO / 'tests' / 'golden' / 'fractal_easy_layout.json'
CKPT = Path('/root/reference/fractal_experiments/frala_easy_final/final_fractal_agent.pt')

DEMO_ARCHS = [   # comprehensive_demo.py:26-58 and its printed parameter counts (:340, :347, :354)
    (dict(input_dim=8, embed_dim=128, num_levels=2, heads=4, share_weights=True), 610_176),
    (dict(input_dim=8, embed_dim=256, num_levels=3, heads=8), 5_912_832),
    (dict(input_dim=8, embed_dim=512, num_levels=4, heads=12, use_hypernetwork=True), 12_342_272),
]


@pytest.mark.parametrize('cfg,count', DEMO_ARCHS)
def test_parameter_count_kat(cfg, count):
    from xtrl_amd.fractal import FractalEncoder
    enc = FractalEncoder(**cfg)
    assert sum(p.numel() for p in enc.parameters()) == count
    assert FR.param_count_encoder(**cfg) == count


def _easy_model():
    from xtrl_amd.fractal import FractalWorldModelActorCritic
    g = json.loads(GOLDEN.read_text())
    fc, ac = g['fractal_config'], g['agent_config']
    heads = fc['fractal_heads']
    dim_head = g['layout']['fractal_encoder.fractal_block.self_attn.to_q.weight'][0] // heads
    wm = FractalWorldModelActorCritic(ac['state_dim'], ac['num_actions'], 100, tuple(ac['reward_range']),
                                      embed_dim=fc['fractal_embed_dim'], num_fractal_levels=fc['num_fractal_levels'],
                                      heads=heads, dim_head=dim_head, fractal_share_weights=fc['fractal_share_weights'],
                                      fractal_use_hypernetwork=fc['fractal_use_hypernetwork'],
                                      continuous_actions=ac['continuous_actions'], evolutionary=ac['evolutionary'])
    return wm, g


def test_checkpoint_layout_matches_reference():
    """Our module tree has exactly the committed checkpoint's parameter names and shapes."""
    wm, g = _easy_model()
    ours = {k: list(v.shape) for k, v in wm.state_dict().items()}
    assert ours == g['layout']


@pytest.mark.skipif(not CKPT.exists(), reason='reference checkpoint only in the build container')
def test_checkpoint_loads_strict():
    wm, g = _easy_model()
    ck = torch.load(CKPT, weights_only=True, map_location='cpu')
    wm.load_state_dict(ck['world_model'], strict=True)
    for k, v in wm.state_dict().items():
        assert abs(float(v.double().sum()) - g['sums'][k]) <= 1e-9 * max(1.0, abs(g['sums'][k])), k
    # the oracle runs on the trained weights
    sd = {k: v.double() for k, v in ck['world_model'].items()}
    x = torch.randn(2, 5, 8, dtype=torch.float64, generator=torch.Generator().manual_seed(0))
    raw, val, _, _, levels = FR.world_model_forward(sd, x, 2, 4, g['layout'][
        'fractal_encoder.fractal_block.self_attn.to_q.weight'][0] // 4, share_weights=True, pre=None)
    assert raw.shape == (2, 4) and val.shape == (2, 100) and len(levels) == 2
    assert torch.isfinite(raw).all() and torch.isfinite(val).all()


def test_one_token_cross_attention_is_value_projection():
    """The HIP path computes the cross-attention to the one-token global state as W_out W_v g (the
    softmax over a single key is exactly 1): check the oracle's full attention agrees."""
    gen = torch.Generator().manual_seed(1)
    d, H, dh = 32, 4, 8
    sd = {f'a.{n}.weight': torch.randn(H * dh if n != 'to_out' else d, d if n != 'to_out' else H * dh,
                                       dtype=torch.float64, generator=gen) for n in ('to_q', 'to_k', 'to_v', 'to_out')}
    x = torch.randn(3, 7, d, dtype=torch.float64, generator=gen)
    g = torch.randn(3, 1, d, dtype=torch.float64, generator=gen)
    full = FR._attention(x, g, sd, 'a', H, dh)
    simple = (g @ sd['a.to_v.weight'].T @ sd['a.to_out.weight'].T).expand_as(full)
    torch.testing.assert_close(full, simple, rtol=1e-12, atol=1e-12)


# ----------------------------------------------------------------------------------------------
# GPU: HIP forward vs the oracle
# ----------------------------------------------------------------------------------------------

def _rand_init(module, seed):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in module.named_parameters():
            scale = 1.0 / math.sqrt(p.shape[-1]) if p.ndim > 1 else 0.3
            is_norm = '.norm' in name and name.endswith('weight')
            p.copy_(torch.randn(p.shape, generator=g) * scale + (1.0 if is_norm else 0.0))


CASES = [   # (embed, levels, heads, dim_head, share, hyper, b, n, ragged)
    (128, 2, 4, 32, True, False, 4, 16, False),
    (256, 3, 8, 32, False, False, 3, 37, True),
    (192, 4, 12, 16, False, True, 2, 70, False),
    (512, 2, 8, 64, False, False, 2, 9, True),
]


@pytest.mark.gpu
@pytest.mark.parametrize('embed,levels,heads,dh,share,hyper,b,n,ragged', CASES)
def test_fractal_encoder_matches_oracle(embed, levels, heads, dh, share, hyper, b, n, ragged):
    from xtrl_amd.fractal import FractalEncoder
    enc = FractalEncoder(8, embed, levels, heads, dh, share_weights=share, use_hypernetwork=hyper)
    _rand_init(enc, embed + n)
    enc = enc.cuda()
    gen = torch.Generator().manual_seed(n)
    x = torch.randn(b, n, 8, generator=gen)
    mask = None
    if ragged:
        lens = torch.randint(1, n + 1, (b,), generator=gen)
        lens[0] = n
        mask = torch.arange(n)[None] < lens[:, None]
    agg, lv = enc(x.cuda(), mask=None if mask is None else mask.cuda(), return_all_levels=True)
    torch.cuda.synchronize()
    sd = {k: v.detach().double().cpu() for k, v in enc.state_dict().items()}
    ref, ref_lv = FR.encoder_forward(sd, x.double(), levels, heads, dh, share, hyper, key_mask=mask, pre='')
    scale = float(ref.abs().max())
    assert float((agg.double().cpu() - ref).abs().max()) <= 1e-4 * scale + 1e-6
    for a, r in zip(lv, ref_lv):
        assert float((a.double().cpu() - r).abs().max()) <= 1e-4 * float(r.abs().max()) + 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize('cont,evo', [(False, False), (False, True), (True, False)])
def test_fractal_world_model_matches_oracle(cont, evo):
    from xtrl_amd.fractal import FractalWorldModelActorCritic
    S, A, b, n = 8, 4, 5, 12
    wm = FractalWorldModelActorCritic(S, A, 100, (-5., 5.), embed_dim=128, num_fractal_levels=2, heads=4, dim_head=32,
                                      continuous_actions=cont, evolutionary=evo, dim_latent_gene=16 if evo else None,
                                      fractal_share_weights=True)
    _rand_init(wm, 7)
    wm = wm.cuda()
    gen = torch.Generator().manual_seed(3)
    state = torch.randn(b, n, S, generator=gen)
    nxt = torch.randn(b, A, generator=gen) if cont else torch.tensor([0, 3, -1, 2, 1])
    gene = torch.randn(b, 16, generator=gen) if evo else None
    out = wm(state.cuda(), next_actions=nxt.cuda(), latent_gene=None if gene is None else gene.cuda())
    torch.cuda.synchronize()
    sd = {k: v.detach().double().cpu() for k, v in wm.state_dict().items()}
    ref = FR.world_model_forward(sd, state.double(), 2, 4, 32, share_weights=True,
                                 next_actions=nxt.double() if cont else nxt, continuous=cont,
                                 latent_gene=None if gene is None else gene.double(), pre=None)
    for name, a, r in zip(('raw_actions', 'values', 'state_pred', 'dones'), out[:4], ref[:4]):
        err = float((a.double().cpu() - r).abs().max())
        assert err <= 1e-4 * float(r.abs().max()) + 1e-6, (name, err)
    for a, r in zip(out[4]['fractal_levels'], ref[4]):
        assert float((a.double().cpu() - r).abs().max()) <= 1e-4 * float(r.abs().max()) + 1e-6


# ----------------------------------------------------------------------------------------------
# the causal fractal policy body (Agent(policy_body='fractal')): host-side checks
# ----------------------------------------------------------------------------------------------

def _policy_pair(levels=2, cont=False, evo=False, dim=32):
    from oracle import ref_port as R
    from xtrl_amd.fractal import FractalPolicyActorCritic
    from xtrl_amd.model import ModelConfig
    c = ModelConfig(state_dim=8, num_actions=4, dim=dim, depth=levels, heads=4, dim_head=8, continuous=cont,
                    evolutionary=evo, dim_gene=8 if evo else 0, reward_range=(-2., 2.))
    mc = R.ModelConfig(8, 4, dim, levels, 4, 8, 100, (-2., 2.), 100, cont, True, evo, 8 if evo else 0)
    return FractalPolicyActorCritic(c, levels), FR.OracleFractalPolicy(mc, levels)


@pytest.mark.parametrize('cont,evo', [(False, False), (True, True)])
def test_policy_body_keeps_reference_names_and_oracle_layout(cont, evo):
    """The Learner's fractal body is FractalWorldModelActorCritic's module tree (reference names,
    separate blocks per level): its state_dict equals the reference class's and the oracle's."""
    from xtrl_amd.fractal import FractalWorldModelActorCritic
    ours, orc = _policy_pair(3, cont, evo)
    ref = FractalWorldModelActorCritic(8, 4, 100, (-2., 2.), embed_dim=32, num_fractal_levels=3, heads=4, dim_head=8,
                                       continuous_actions=cont, evolutionary=evo, dim_latent_gene=8 if evo else None)
    shapes = lambda m: {k: tuple(v.shape) for k, v in m.state_dict().items()}   # noqa: E731
    assert shapes(ours) == shapes(ref) == shapes(orc)
    assert sorted(ours.flat_order()) == sorted(n for n, _ in ours.named_parameters())


def test_policy_oracle_streaming_equals_whole_sequence_and_is_causal():
    """Position t of the oracle depends on states 0..t only, and running it position by position
    with the cache equals one call over the sequence (the rollout's and the learn step's views)."""
    _, orc = _policy_pair(2, evo=True)
    _rand_init(orc, 4)
    g = torch.Generator().manual_seed(5)
    st = torch.randn(3, 9, 8, generator=g, dtype=torch.float64)
    lat = torch.randn(3, 8, generator=g, dtype=torch.float64)
    orc = orc.double()
    raw, val, *_ = orc(st, latent_gene=lat)
    cache, outs = None, []
    for t in range(9):
        r, _, _, _, cache = orc(st[:, t:t + 1], latent_gene=lat, cache=cache)
        outs.append(r)
    torch.testing.assert_close(torch.cat(outs, 1), raw, rtol=1e-12, atol=1e-12)
    st2 = st.clone()
    st2[:, 5:] += 1.0                      # the future changes, the past does not
    raw2, val2, *_ = orc(st2, latent_gene=lat)
    torch.testing.assert_close(raw2[:, :5], raw[:, :5], rtol=0, atol=0)
    torch.testing.assert_close(val2[:, :5], val[:, :5], rtol=0, atol=0)
    assert float((raw2[:, 5:] - raw[:, 5:]).abs().max()) > 1e-3


def test_policy_body_rejects_decoder_only_options():
    from xtrl_amd import Learner
    with pytest.raises(NotImplementedError):
        Learner(state_dim=8, num_actions=4, reward_range=(-1., 1.), batch_size=2, num_episodes_per_update=2,
                world_model=dict(attn_dim_head=16, heads=4, depth=2, attn_gate_values=True),
                agent_kwargs=dict(policy_body='fractal'))
