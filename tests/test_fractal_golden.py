"""Pin oracle/fractal_ref.py against the reference's OWN fractal modules (CPU).

tests/golden/fractal.npz comes from tests/golden/make_golden.py, which executes
x_transformers_rl/fractal_rl.py in the build container with x-transformers' Attention / FeedForward
restated (oracle/thirdparty.py XAttention / FeedForward).  So these fixtures pin the reference's
own arithmetic — level embedding (learned + sinusoidal scale, fractal_rl.py:50-67), the post-norm
block order (:120-132), the global-state update (:315-317), the level projections + mean pooling and
final aggregation (:329-341), the world-model / actor / critic heads (:570-619) — while the
x-transformers attention internals stay the restatement's.  The causal per-timestep policy body the
Learner trains (OracleFractalPolicy) is pinned at its first position, where causal and the
reference's sequence-pooled forward coincide exactly (one token: softmax over one key, means over one
position)."""
import numpy as np
import pytest
import torch

from oracle import fractal_ref as FR
from oracle import ref_port as R


@pytest.fixture(scope='module')
def fx(golden):
    return golden('fractal')


def sd_of(fx, prefix):
    """The state_dict stored under ``prefix`` (inputs / outputs of the case excluded)."""
    data = {'x', 'g', 'mask', 'out', 'out_nomask', 'out_noglobal', 'agg', 'levels'}
    return {k[len(prefix):]: torch.from_numpy(fx[k]) for k in fx.files if k.startswith(prefix)
            and k[len(prefix):] not in data and not k[len(prefix):].startswith(('n8.', 'n1.'))}


def T(a):
    return torch.from_numpy(np.asarray(a))


def close(a, b, tol=2e-6):
    """fp32 on both sides (the fixtures are the reference's fp32 outputs): max error relative to the
    output's scale."""
    b = T(b).double()
    scale = max(float(b.abs().max()), 1e-30)
    err = float((a.double() - b).abs().max())
    assert err <= tol * scale, err / scale


def test_level_embedding(fx):
    sd = sd_of(fx, 'le.')
    close(sd['level_embeds'] + sd['scale_embeds'], fx['le.out'])
    # the oracle's sinusoidal scale table (used by OracleFractalPolicy) is the reference's buffer
    torch.testing.assert_close(FR._OLevelEmb(5, 24).scale_embeds, torch.from_numpy(fx['le.scale_embeds']),
                               rtol=0, atol=1e-6)


def test_processing_block(fx):
    sd = sd_of(fx, 'blk.')
    x, g, m = T(fx['blk.x']), T(fx['blk.g']), T(fx['blk.mask'])
    sdd = {'.' + k: v for k, v in sd.items()}
    close(FR._block(x, g, sdd, '', 4, 8, m), fx['blk.out'])
    close(FR._block(x, g, sdd, '', 4, 8), fx['blk.out_nomask'])
    close(FR._block(x, None, sdd, '', 4, 8, m), fx['blk.out_noglobal'])


@pytest.mark.parametrize('tag,share,hyper', [('sep', False, False), ('share', True, False), ('hyper', False, True)])
def test_encoder(fx, tag, share, hyper):
    sd = sd_of(fx, f'enc_{tag}.')
    x = T(fx['enc.x'])
    mask = T(fx['enc.mask']) if tag == 'sep' else None
    agg, levels = FR.encoder_forward(sd, x, 3, 4, 8, share, hyper, key_mask=mask, pre='')
    close(agg, fx[f'enc_{tag}.agg'])
    close(torch.stack(levels), fx[f'enc_{tag}.levels'])


@pytest.mark.parametrize('tag,cont,evo', [('wm_d', False, True), ('wm_c', True, False)])
@pytest.mark.parametrize('n', [8, 1])
def test_world_model_forward(fx, tag, cont, evo, n):
    sd = sd_of(fx, f'{tag}.')
    p = f'{tag}.n{n}.'
    lat = T(fx[p + 'latent']) if evo else None
    raw, val, sp, dn, levels = FR.world_model_forward(sd, T(fx[p + 'state']), 2, 4, 8, next_actions=T(fx[p + 'next_actions']),
                                                      latent_gene=lat, continuous=cont, pre=None)
    for name, a in (('raw', raw), ('values', val), ('state_pred', sp), ('dones', dn)):
        close(a, fx[p + name])
    close(torch.stack(levels), fx[p + 'levels'])


@pytest.mark.parametrize('tag,cont,evo', [('wm_d', False, True), ('wm_c', True, False)])
def test_causal_policy_first_position_is_reference_forward(fx, tag, cont, evo):
    """OracleFractalPolicy (the causal body the Learner trains) at t = 0 equals the reference's
    FractalWorldModelActorCritic.forward on the one-position sequence, on the reference's weights."""
    mc = R.ModelConfig(6, 4, 32, 2, 4, 8, 16, (-2., 2.), 100, cont, cont, evo, 8 if evo else 0)
    pol = FR.OracleFractalPolicy(mc, 2).eval()
    pol.load_state_dict({k: v for k, v in sd_of(fx, f'{tag}.').items()}, strict=True)
    p = f'{tag}.n1.'
    nxt = T(fx[p + 'next_actions'])
    lat = T(fx[p + 'latent']) if evo else None
    with torch.no_grad():
        raw, val, sp, dn, _ = pol(T(fx[p + 'state']), next_actions=nxt[:, None] if not cont else nxt[:, None, :],
                                  latent_gene=lat)
    close(raw[:, 0], fx[p + 'raw'])
    close(val[:, 0], fx[p + 'values'])
    close(sp[:, :, 0], fx[p + 'state_pred'])
    close(dn[:, 0], fx[p + 'dones'])
