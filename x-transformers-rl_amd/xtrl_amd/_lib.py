"""ctypes binding of libxtrl_hip.so (include/xtrl_hip.h).

The library is the product's compute path.  There is no CPU fallback: if the shared object is
missing or no MI355X is visible, every compute call raises.  ``load()`` itself only needs the file
(the CPU test-suite checks the exported symbols without running kernels).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import torch   # noqa: F401  (load torch's HIP runtime first so the library binds to the same one)

LIB_PATH = Path(os.environ.get('XTRL_LIB', Path(__file__).resolve().parent / 'libxtrl_hip.so'))   # override: A/B experiments
ABI_VERSION = 21

P = C.c_void_p
I32, I64, U32, U64, F32 = C.c_int, C.c_int64, C.c_uint32, C.c_uint64, C.c_float

ACT_NONE, ACT_GELU, ACT_SILU, ACT_RELU = 0, 1, 2, 3

# stats[] slots of the fused loss (XTRL_LS_*)
LS = dict(loss=0, actor=1, critic=2, autoreg=3, done=4, adv_mean=5, adv_den=6, L=7, Lc=8, nmask=9, nwm=10,
          kcrit=11, dL=12, dLc=13)
LOSS_TOK, LOSS_STATS = 30, 32


class DecodeLayer(C.Structure):
    _fields_ = [(n, P) for n in ('ln_attn', 'w_qkv', 'b_qkv', 'w_out', 'ln_ff', 'w_ff1', 'b_ff1', 'w_ff2', 'b_ff2',
                                 'k_cache', 'v_cache', 'w_out_t', 'w_ff1x', 'w_ff2x', 'w_qkv_t', 'w_ff1_t', 'w_ff2_t',
                                 'w_ff1f', 'w_ff2f')]


class RngState(C.Structure):
    _fields_ = [('seed', U64), ('update', U32), ('slot_offset', U32)]


class DecodeDesc(C.Structure):
    _fields_ = ([(n, I32) for n in ('E', 'S', 'A', 'B', 'd', 'L', 'H', 'dh', 'Tmax', 'G', 'ff', 'in_dim', 'n_qkv',
                                    'continuous', 'squash', 'evolutionary', 'gate_values', 'value_residual',
                                    'learned_mix', 'rotary_abs', 'rot_dim', 'sim_mode', 'hazard_log2', 'no_reward_cond',
                                    'state_only')]
                + [('rs_eps', F32), ('clamp_lo', F32), ('clamp_hi', F32), ('has_clamp', I32)]
                + [(n, P) for n in ('w_pin', 'b_pin', 'act_emb', 'act_emb_b', 'reward_embed', 'w_se', 'b_se',
                                    'ln_final', 'w_h1', 'b_h1', 'w_h2', 'b_h2', 'inv_freq')]
                + [('layers', C.POINTER(DecodeLayer))]
                + [(n, P) for n in ('rs_mean', 'rs_var', 'state', 'prev_action', 'prev_action_f', 'prev_reward',
                                    'alive', 'lens', 'cum_reward', 'episode_of_slot', 'slot_of_row', 'rng', 'traj_states',
                                    'traj_actions', 'traj_actions_f', 'traj_logp', 'traj_rewards', 'traj_bounds',
                                    'traj_values', 'x', 'qkv', 'att', 'hff', 'ac_in', 'logits', 'v1', 'xn', 'live_rows', 'live_count',
                                    'mlp_part', 'mlp_cnt', 'lat_embed')]
                + [('prof_events', C.POINTER(C.c_void_p))]
                + [(n, P) for n in ('w_h1_t', 'w_h2_t')]
                + [('layers_dev', C.POINTER(DecodeLayer))]
                + [(n, P) for n in ('w_h1x', 'heads_part', 'heads_cnt', 'row_part', 'row_cnt')]
                + [('ff_glu', I32), ('hglu', P), ('qk_norm', I32), ('attn_scale', F32), ('xpos_base', F32),
                   ('rms_norm', I32), ('act_host', P)])


class FractalLevel(C.Structure):
    _fields_ = [(n, P) for n in ('w_qkv', 'w_out', 'ln1_w', 'ln1_b', 'w_c', 'ln2_w', 'ln2_b', 'w_ff1', 'b_ff1',
                                 'w_ff2', 'b_ff2', 'ln3_w', 'ln3_b', 'w_pg', 'b_pg', 'level_emb', 'sums')]


class FractalDesc(C.Structure):
    _fields_ = ([('levels', I32), ('ln_eps', F32), ('level', C.POINTER(FractalLevel))]
                + [(n, P) for n in ('g_init', 'c0', 'w_fa0', 'b_fa0', 'w_fa2', 'b_fa2', 'g', 'c2', 'tmp', 'x2', 'mean',
                                    'allf', 'hagg')])


class LossDesc(C.Structure):
    _fields_ = ([(n, I32) for n in ('b', 'n', 'A', 'B', 'S1', 'continuous', 'squash', 'hl_reduction_mean')]
                + [(n, F32) for n in ('eps_clip', 'value_clip', 'entropy_weight', 'w_actor', 'w_critic', 'w_autoreg',
                                      'lo', 'hi', 'sigma')]
                + [(n, P) for n in ('raw_actions', 'values', 'pred_raw', 'done_logit', 'actions', 'actions_f',
                                    'old_logp', 'returns', 'old_values', 'dones', 'lens', 'real', 'support', 'centers',
                                    'tok', 'stats', 'd_raw_actions', 'd_values', 'd_pred_raw', 'd_done_logit')])


class TrainLayer(C.Structure):
    _fields_ = ([(n, I64) for n in ('ln_attn', 'w_proj', 'b_proj', 'w_out', 'ln_ff', 'w_ff1', 'b_ff1', 'w_ff2',
                                    'b_ff2')]
                + [('n_qkv', I32), ('mix', I32)]
                + [(n, P) for n in ('x_attn', 'x_ff', 'xn_attn', 'xn_ff', 'st_attn', 'st_ff', 'proj', 'qkv', 'o', 'og',
                                    'lse', 'u', 'hd')])


class TrainDesc(C.Structure):
    _fields_ = ([(n, I32) for n in ('b', 'n', 'S', 'A', 'd', 'L', 'H', 'dh', 'ff', 'B', 'in_dim', 'n_out', 'G',
                                    'continuous', 'evolutionary', 'gate_values', 'rot_dim')]
                + [(n, F32) for n in ('dropout', 'frac_head_grad', 'reward_keep', 'attn_scale')]
                + [('seed', U64), ('attn_offset', U32), ('ff_offset', U32), ('flat', P), ('grad', P)]
                + [(n, I64) for n in ('w_pin', 'act_emb', 'act_emb_b', 'reward_embed', 'w_se', 'b_se', 'ln_final',
                                      'w_pd', 'b_pd', 'w_pred2', 'b_pred2', 'w_lat', 'b_lat', 'w_h1', 'b_h1', 'w_a2',
                                      'b_a2', 'w_c2', 'b_c2')]
                + [(n, P) for n in ('inv_freq', 'swr', 'prev_action', 'next_action', 'prev_action_f',
                                    'next_action_f', 'latent', 'lens', 'raw', 'values', 'pred', 'done', 'x_final',
                                    'st_final', 'ac_in', 'ewa', 'zp', 'hp', 'z1', 'h1', 'lat_e', 'd_raw', 'd_values',
                                    'd_pred', 'd_done', 'dx', 'dx2', 'dxn', 'dff', 'dproj', 'dog', 'dvfirst', 'dz1', 'dac',
                                    'dzp', 'dewa', 'delta', 'part')]
                + [('part_floats', I64), ('ws', P), ('ws_floats', I64), ('layers', C.POINTER(TrainLayer)),
                   ('prof_events', C.POINTER(C.c_void_p)), ('prof_flops', P), ('prof_cap', I32), ('prof_n', P),
                   ('grad_events', C.POINTER(C.c_void_p)), ('ld_ff', I32),
                   ('scratch_per_layer', I32), ('ff_glu', I32), ('ld_u2', I32), ('glu_dh', P),
                   ('qk_norm', I32), ('xpos_base', F32), ('rms_norm', I32),
                   ('Tv', I32), ('vrows', P), ('vinv', P), ('ewa_v', P), ('hp_v', P), ('zp_v', P), ('pred_v', P),
                   ('d_pred_v', P), ('dzp_v', P), ('dewa_v', P), ('dq_part', P), ('dq_part_floats', I64),
                   ('packed', I32), ('ep_off', P), ('pack_ws', P), ('pack_ws_floats', I64)])


class FractalTrainLevel(C.Structure):
    _fields_ = ([(n, I64) for n in ('w_qkv', 'w_out', 'w_gv', 'w_go', 'ln1_w', 'ln1_b', 'ln2_w', 'ln2_b', 'ln3_w',
                                    'ln3_b', 'w_ff1', 'b_ff1', 'w_ff2', 'b_ff2', 'w_proj', 'b_proj', 'level_embed')]
                + [(n, P) for n in ('xin', 'qkv', 'o', 'lse', 's1', 'x1', 'st1', 'g', 'gv', 's2', 'x2', 'st2', 'h', 'u',
                                    's3', 'x3', 'st3', 'mean')])


class FractalTrainDesc(C.Structure):
    _fields_ = ([('levels', I32)]
                + [(n, I64) for n in ('b_in', 'g_init', 'w_gu', 'b_gu', 'w_fa0', 'b_fa0', 'w_fa2', 'b_fa2')]
                + [(n, P) for n in ('scale_embeds', 'le', 'bias0', 'cat', 'hfa', 'dxa', 'dxb', 'dmean', 'ds',
                                    'dga', 'dgb', 'dgv', 'dz', 'dqkv', 'dob', 'dcat', 'dhfa')]
                + [('level', C.POINTER(FractalTrainLevel))])


class BatchDesc(C.Structure):
    _fields_ = ([(n, I32) for n in ('N', 'Tmax', 'n', 'b', 'S', 'A', 'B', 'continuous')]
                + [(n, P) for n in ('states', 'actions', 'actions_f', 'rewards', 'logp', 'bounds', 'values', 'returns',
                                    'lens', 'idx', 'rs_mean', 'rs_var', 'swr', 'prev_action', 'action',
                                    'prev_action_f', 'action_f', 'old_logp', 'mb_returns', 'old_values', 'dones',
                                    'mb_lens', 'rs_part', 'rs_m')])


SIGNATURES = {
    'xtrl_abi_version': (I32, []),
    'xtrl_struct_size': (C.c_int64, [C.c_char_p]),
    'xtrl_last_error': (C.c_char_p, []),
    'xtrl_gemm_f32': (I32, [P, I32, P, I32, P, P, P, I32, P, I32, P, I64, I32, I32, I32, I32, P]),
    'xtrl_gemm_ex': (I32, [I32, I32, P, I32, P, I32, P, P, I32, I32, I32, I32, F32, P]),
    'xtrl_gemm_wgrad': (I32, [P, I32, P, I32, P, I32, I32, I32, I32, F32, P, I64, P]),
    'xtrl_gemm_wgrad_db': (I32, [P, I32, P, I32, P, I32, I32, I32, I32, F32, P, I64, P, I32, P]),
    'xtrl_linear_gelu_drop': (I32, [P, I32, P, P, P, I32, P, I32, I32, I32, I32, F32, U64, U32, U32, P]),
    'xtrl_layernorm_f32': (I32, [P, I32, P, P, I32, I32, I32, P]),
    'xtrl_rollout_begin': (I32, [C.POINTER(DecodeDesc), P]),
    'xtrl_decode_step': (I32, [C.POINTER(DecodeDesc), I32, P]),
    'xtrl_decode_step_rows': (I32, [C.POINTER(DecodeDesc), I32, I32, P]),
    'xtrl_row_stamps': (I32, [I32, P, I32, P]),
    'xtrl_host_decode': (I32, [C.POINTER(DecodeDesc), I32, I32, P, P]),
    'xtrl_host_feedback': (I32, [C.POINTER(DecodeDesc), I32, P, P, I32, I32, P]),
    'xtrl_rollout_env_feedback': (I32, [C.POINTER(DecodeDesc), I32, P, P, P, P, I32, I32, P]),
    'xtrl_host_row_step': (I32, [C.POINTER(DecodeDesc), I32, P, I32, I32, P, P]),
    'xtrl_host_wait': (I32, [P, C.c_uint32, C.c_double]),
    'xtrl_dgemm': (I32, [P, I32, P, P, P, I32, P, I32, P, I32, P, P, I32, I32, I32, I32, P]),
    'xtrl_dgemm_pack': (I32, [P, I32, I32, I32, P, P]),
    'xtrl_fractal_decode_step': (I32, [C.POINTER(DecodeDesc), C.POINTER(FractalDesc), I32, P]),
    'xtrl_dgemm_packed_floats': (I64, [I32, I32]),
    'xtrl_dgemm_pack_x6': (I32, [P, I32, I32, I32, P, P]),
    'xtrl_dgemm_packed_x6_elems': (I64, [I32, I32]),
    'xtrl_dgemm_pack_f8': (I32, [P, I32, I32, I32, P, P]),
    'xtrl_glu_drop_fwd': (I32, [P, I32, P, I32, I32, I32, F32, U64, U32, U32, P]),
    'xtrl_glu_drop_bwd': (I32, [P, I32, P, I32, P, I32, I32, I32, F32, U64, U32, U32, P]),
    'xtrl_dgemm_packed_f8_floats': (I64, [I32, I32]),
    'xtrl_hlgauss_gae': (I32, [P, I64, P, P, I64, P, P, P, I32, I32, I32, F32, F32, P, P, P]),
    'xtrl_attn_fwd': (I32, [P, P, P, P, P, P, I32, I32, I32, I32, F32, F32, U64, U32, U32, P]),
    'xtrl_attn_bwd': (I32, [P, P, P, P, P, P, P, P, P, P, P, I32, I32, I32, I32, F32, F32, U64, U32, U32, P]),
    'xtrl_attn_bwd_part_floats': (I64, [I32, I32, I32, I32]),
    'xtrl_train_pack_floats': (I64, [I32, I32, I32, I32, I32]),
    'xtrl_attn_bwd_part': (I32, [P, P, P, P, P, P, P, P, P, P, P, P, I64, I32, I32, I32, I32, F32, F32, U64, U32, U32,
                                  P]),
    'xtrl_loss_fwd': (I32, [C.POINTER(LossDesc), P]),
    'xtrl_loss_bwd': (I32, [C.POINTER(LossDesc), F32, P]),
    'xtrl_grad_norm': (I32, [P, I64, P, F32, P, P]),
    'xtrl_adopt_atan2': (I32, [P, P, P, P, P, I64, P, I32, P, I32, P, P, F32, F32, F32, F32, F32, F32, F32, F32, F32,
                               I32, P]),
    'xtrl_ema_lerp': (I32, [P, P, I64, F32, P]),
    'xtrl_sim_reset': (I32, [P, I32, I32, U64, U32, P, P]),
    'xtrl_train_forward': (I32, [C.POINTER(TrainDesc), P]),
    'xtrl_train_backward': (I32, [C.POINTER(TrainDesc), P]),
    'xtrl_ff_dropout_mask': (I32, [P, I32, I32, F32, U64, U32, U32, P]),
    'xtrl_train_part_floats': (C.c_int64, [I32, I32, I32, I32]),
    'xtrl_minibatch_gather': (I32, [C.POINTER(BatchDesc), P]),
    'xtrl_rsnorm_update': (I32, [P, P, P, I32, I32, P]),
    'xtrl_attn_fwd_tokens': (I32, [P, I32, P, I32, P, I32, P, P, I32, P, I32, I32, I32, I32, F32, I32, P]),
    'xtrl_rows_add': (I32, [P, I32, P, P, I32, I32, I32, P]),
    'xtrl_add_layernorm': (I32, [P, I32, P, I32, I32, P, P, P, I32, I32, I32, F32, P]),
    'xtrl_seq_mean': (I32, [P, I32, I32, I32, I32, P, I32, P]),
    'xtrl_safe_embed': (I32, [P, I32, P, I32, P, I32, P]),
    'xtrl_wm_post': (I32, [P, I32, I32, I32, P, P, I32, P, P]),
    'xtrl_rng_uniform': (F32, [U64, U32, U32, U32, U32, U32]),
    'xtrl_rng_normal': (F32, [U64, U32, U32, U32, U32, U32]),
    'xtrl_source_hash': (C.c_char_p, []),
    'xtrl_fractal_train_forward': (I32, [C.POINTER(TrainDesc), C.POINTER(FractalTrainDesc), P]),
    'xtrl_fractal_train_backward': (I32, [C.POINTER(TrainDesc), C.POINTER(FractalTrainDesc), P]),
}

STRUCTS = {'XtrlDecodeLayer': DecodeLayer, 'XtrlRngState': RngState, 'XtrlDecodeDesc': DecodeDesc,
           'XtrlTrainLayer': TrainLayer, 'XtrlTrainDesc': TrainDesc, 'XtrlBatchDesc': BatchDesc,
           'XtrlLossDesc': LossDesc, 'XtrlFractalLevel': FractalLevel, 'XtrlFractalDesc': FractalDesc,
           'XtrlFractalTrainLevel': FractalTrainLevel, 'XtrlFractalTrainDesc': FractalTrainDesc}

_lib = None


def load():
    """Load and declare the library (no GPU needed)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(f'{LIB_PATH} is missing: build it with `make -C x-transformers-rl_amd` '
                               f'or __graft_entry__.build() (the MI355X path has no CPU fallback)')
        lib = C.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        if lib.xtrl_abi_version() != ABI_VERSION:
            raise RuntimeError(f'libxtrl_hip ABI {lib.xtrl_abi_version()} != {ABI_VERSION}')
        from ._srchash import source_hash
        built, here = lib.xtrl_source_hash().decode(), source_hash()
        # (an explicit XTRL_LIB — A/B experiments against a saved build — is taken as chosen)
        if built != here and 'XTRL_LIB' not in os.environ:   # compiled from other sources than this tree's
            raise RuntimeError(f'{LIB_PATH} was built from sources {built}, the tree holds {here}: rebuild it '
                               f'with `make -C x-transformers-rl_amd` or __graft_entry__.build()')
        for cname, py in STRUCTS.items():   # a stale build against an edited header fails here
            got = lib.xtrl_struct_size(cname.encode())
            if got != C.sizeof(py):
                raise RuntimeError(f'libxtrl_hip {cname} is {got} bytes, the binding {C.sizeof(py)}: rebuild')
        _lib = lib
    return _lib


def lib():
    """The library, for a compute call: requires an MI355X."""
    if not torch.cuda.is_available():
        raise RuntimeError('xtrl_amd needs a ROCm GPU (gfx950); no CPU fallback exists by design')
    return load()


def check(rc, what=''):
    if rc != 0:
        msg = load().xtrl_last_error().decode(errors='replace')
        raise RuntimeError(f'libxtrl_hip {what} failed (code {rc}): {msg}')


def ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def rng_uniform(seed, update, slot, t, field, sub=0):
    return load().xtrl_rng_uniform(seed & 0xFFFFFFFFFFFFFFFF, update, slot, t, field, sub)


FIELD_STATE, FIELD_REWARD, FIELD_TERM, FIELD_SAMPLE, FIELD_COIN, FIELD_DROPOUT, FIELD_FF_DROPOUT = 1, 2, 3, 4, 5, 6, 7
