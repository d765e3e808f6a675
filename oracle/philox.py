"""Counter-based random streams + the synthetic LunarLander-shaped Sim — TEST INFRASTRUCTURE ONLY.

numpy restatement of x-transformers-rl_amd/csrc/philox.h (the HIP side).  Both sides must agree
bit for bit, so everything is integer arithmetic plus a fixed-order sequence of f32 adds / one f32
multiply (no transcendental functions, no FMA-contractible expressions):

  philox4x32-10(counter = (c0, c1, c2, c3), key = (seed_lo, seed_hi))
  counter layout:  c0 = slot/env/minibatch, c1 = timestep/epoch, c2 = learning update,
                   c3 = (field << 24) | sub-index
  uniform(x)    = (x >> 8) * 2^-24                                   in [0, 1), exact in f32
  normal(block) = (((u0 + u1) + u2) + u3 - 2) * sqrt(3)   (f32)      Irwin-Hall(4), var 1

The synthetic Sim (SURVEY §8d / BASELINE.md inputs):
  'readme'  state ~ N(0,1)^S, reward ~ N(0,1), never terminates      (README Sim, config C1)
  'lander'  state ~ N(0,1)^S, reward ~ N(0,1) * (1 + 0.1 a), terminated with hazard 2^-hazard_log2
            per step (default 1/64)                                   (configs C2-C5)
Streams are keyed by the *episode* index so every gene of an EPO population sees the same env
realisation, as the reference does by reusing episode seeds across genes (xtrl.py:1216-1228).
"""
from __future__ import annotations

import numpy as np
import torch

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

FIELD_STATE = 1
FIELD_REWARD = 2
FIELD_TERM = 3
FIELD_SAMPLE = 4
FIELD_COIN = 5
FIELD_DROPOUT = 6
FIELD_FF_DROPOUT = 7

SQRT3 = np.float32(1.7320508075688772)


def philox4x32(c0, c1, c2, c3, seed):
    """Vectorised Philox4x32-10; arguments broadcast; returns 4 uint32 arrays."""
    c = [np.asarray(x, dtype=np.uint64) & MASK32 for x in np.broadcast_arrays(c0, c1, c2, c3)]
    k0 = np.uint64(int(seed) & 0xFFFFFFFF)
    k1 = np.uint64((int(seed) >> 32) & 0xFFFFFFFF)
    for _ in range(10):
        p0 = M0 * c[0]
        p1 = M1 * c[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
        k0 = (k0 + np.uint64(W0)) & MASK32
        k1 = (k1 + np.uint64(W1)) & MASK32
    return [x.astype(np.uint32) for x in c]


def to_uniform(x):
    return (x >> np.uint32(8)).astype(np.float32) * np.float32(2.0 ** -24)


def _c3(field, sub):
    return (np.uint64(field) << np.uint64(24)) | (np.asarray(sub, dtype=np.uint64) & np.uint64(0xFFFFFF))


def philox_uniform(seed, update, slot, t, field, count, normal=False):
    """``count`` f32 values for one (slot, t, update, field); element i uses sub-index i."""
    sub = np.arange(count)
    r = philox4x32(slot, t, update, _c3(field, sub), seed)
    if not normal:
        return to_uniform(r[0])
    u = [to_uniform(x) for x in r]
    s = ((u[0] + u[1]) + u[2]) + u[3]
    return ((s - np.float32(2.0)) * SQRT3).astype(np.float32)


def philox_u32(seed, update, slot, t, field, sub=0):
    return philox4x32(slot, t, update, _c3(field, sub), seed)[0]


def epoch_permutation(seed, update, epoch, n):
    """Minibatch order of one epoch (stands in for DataLoader(shuffle=True), xtrl.py:876-878)."""
    g = torch.Generator().manual_seed((int(seed) * 1000003 + int(update)) * 1000003 + int(epoch) & (2 ** 62 - 1))
    return torch.randperm(n, generator=g)


def evolve_seed(seed, update, epoch, minibatch):
    """Global torch seed set right before each LatentGenePool.evolve_ (evo.py:76-184 draws from the
    global torch RNG; pinning it per call makes the EPO step reproducible across implementations)."""
    return ((int(seed) * 7919 + int(update)) * 7919 + int(epoch)) * 7919 + int(minibatch) & (2 ** 62 - 1)


def reward_coin(seed, update, epoch, minibatch, p):
    """All-or-nothing reward-conditioning keep coin of one training forward (xtrl.py:501-503)."""
    if p <= 0.:
        return True
    u = philox_uniform(seed, update, minibatch, epoch, FIELD_COIN, 1)[0]
    return bool(u >= np.float32(p))


REWARD_FACTORS = np.array([np.float32(1.0 + 0.1 * a) for a in range(64)], dtype=np.float32)


class SynthSim:
    """Scalar view of one env lane of the vectorised synthetic Sim (reset/step duck type)."""

    def __init__(self, seed, update, episode, state_dim, num_actions, mode='lander', hazard_log2=6):
        self.seed, self.update, self.episode = seed, update, episode
        self.S, self.A, self.mode, self.hazard_log2 = state_dim, num_actions, mode, hazard_log2
        self.t = 0

    def _state(self, t):
        return philox_uniform(self.seed, self.update, self.episode, t, FIELD_STATE, self.S, normal=True)

    def reset(self, seed=None):
        self.t = 0
        return self._state(0)

    def step(self, action):
        t = self.t
        z = philox_uniform(self.seed, self.update, self.episode, t, FIELD_REWARD, 1, normal=True)[0]
        a = np.asarray(action)
        if self.mode == 'lander' and a.ndim == 0:
            reward = np.float32(z * REWARD_FACTORS[int(a)])
        else:
            reward = np.float32(z)
        terminated = False
        if self.mode == 'lander' and self.hazard_log2 > 0:
            x = philox_u32(self.seed, self.update, self.episode, t, FIELD_TERM)
            terminated = bool((int(x) & ((1 << self.hazard_log2) - 1)) == 0)
        self.t = t + 1
        return self._state(t + 1), reward, terminated


# --------------------------------------------------------------------------------------------
# learn-step dropout keep masks (the streams csrc/attn.hip and the GELU + dropout GEMM epilogue
# of csrc/gemm.hip draw; include/xtrl_hip.h "dropout streams"), so that the oracle's training
# forward can apply the GPU's masks in place of torch.nn.Dropout (x-transformers attn_dropout /
# FeedForward Dropout, xtrl.py:729-730) and be compared with dropout ON
# --------------------------------------------------------------------------------------------


def _thresh32(p):
    return np.uint32(min(int(p * 2 ** 32), 2 ** 32 - 1))


def attn_dropout_keep(b, H, n, p, seed, offset, layer):
    """bool [b][H][n][n] attention keep mask (x-transformers-rl_amd/csrc/attn.hip), c2 = offset + e H + h.
    p a multiple of 1/256 (byte mode): byte (i & 3) of word ((j >> 4) & 3) of philox4x32(i >> 2,
    16 (j >> 6) + (j & 15), c2, FIELD_DROPOUT << 24 | (layer | 1 << 23); seed) >= 256 p (one block per
    4 query rows x 4 keys 16 apart); otherwise word (i & 3) of philox4x32(i >> 2, j, c2,
    FIELD_DROPOUT << 24 | layer; seed) >= p 2^32."""
    n4 = (n + 3) // 4
    c2 = (np.uint64(offset) + np.arange(b * H, dtype=np.uint64))[:, None, None]
    if float(p * 256).is_integer():
        J = 16 * ((n + 63) // 64)
        words = np.stack(philox4x32(np.arange(n4)[None, :, None], np.arange(J)[None, None, :], c2,
                                    _c3(FIELD_DROPOUT, layer | (1 << 23)), seed), axis=1)   # [bH][word][i >> 2][c1]
        i, j = np.arange(n)[:, None], np.arange(n)[None, :]
        w = words[:, (j >> 4) & 3, i >> 2, 16 * (j >> 6) + (j & 15)]                         # [bH][n][n]
        byte = (w >> (8 * (i & 3)).astype(np.uint32)) & np.uint32(0xFF)
        return (byte >= np.uint32(int(p * 256))).reshape(b, H, n, n)
    words = philox4x32(np.arange(n4)[None, :, None], np.arange(n)[None, None, :], c2,
                       _c3(FIELD_DROPOUT, layer), seed)
    w = np.stack(words, axis=2).reshape(b * H, 4 * n4, n)[:, :n]     # row i = 4 (i >> 2) + (i & 3)
    return (w >= _thresh32(p)).reshape(b, H, n, n)


def ff_dropout_keep(M, N, p, seed, offset, layer):
    """bool [M][N] feed-forward keep mask over token-major rows m (= episode * n + step) and hidden
    columns.  p a multiple of 1/256 (byte mode): byte (m & 3) of word ((m >> 3) & 3) of
    philox4x32(col, 2 (m >> 5) + ((m >> 2) & 1), offset, FIELD_FF_DROPOUT << 24 | 2 layer + 1; seed)
    >= 256 p (one block per 16 rows); otherwise word (m & 3) of philox4x32(col, m >> 2, offset,
    FIELD_FF_DROPOUT << 24 | 2 layer; seed) >= p 2^32."""
    m = np.arange(M)
    cols = np.arange(N)[None, :]
    if float(p * 256).is_integer():
        G2 = 2 * ((M + 31) // 32)
        words = np.stack(philox4x32(cols, np.arange(G2)[:, None], offset, _c3(FIELD_FF_DROPOUT, 2 * layer + 1),
                                    seed))                            # [word][c1][col]
        c1 = ((m >> 5) << 1) | ((m >> 2) & 1)
        w = words[(m >> 3) & 3, c1]                                   # [M][N]
        return ((w >> (8 * (m & 3))[:, None].astype(np.uint32)) & np.uint32(0xFF)) >= np.uint32(int(p * 256))
    M4 = (M + 3) // 4
    words = np.stack(philox4x32(cols, np.arange(M4)[:, None], offset, _c3(FIELD_FF_DROPOUT, 2 * layer), seed))
    return words[m & 3, m >> 2] >= _thresh32(p)
