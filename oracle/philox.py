"""Philox4x32-10 and the 23-bit uniform, restated in numpy (test oracle only).

The reference draws its Gumbel noise with ``tf.random_uniform``
(``maddpg/common/distributions.py:264-266``, ``SoftCategoricalPd.sample``),
which TF1 implements as Philox4x32-10 (``tensorflow/core/lib/random/
philox_random.h``: multipliers 0xD2511F53 / 0xCD9E8D57, Weyl key increments
0x9E3779B9 / 0xBB67AE85) followed by a 23-random-bit float in [0, 1)
(``random_distributions.h`` ``Uint32ToFloat``).  The reference never seeds it
(no op or graph seed), so its noise stream is not reproducible and no bit-level
parity with it exists; what can be pinned is the generator itself:

* ``philox4x32_10`` is checked against the Random123 known-answer vectors
  (``KAT``, published with the algorithm: Salmon et al., SC'11) in
  ``tests/test_oracle.py``;
* ``uniforms5`` restates the device's draw (``mdp_device.h`` ``uniforms5``:
  counter (row, ctr, stream, 0|1), key = the 64-bit seed; the float keeps the
  HIGH 23 bits of each word -- TF1 keeps the low 23 -- the same distribution on
  the same 2^-23 grid), and ``tests/test_gpu_parity.py`` compares the device's
  own Gumbel draws (``mdp_act`` without injected uniforms) with it.
"""
import numpy as np

M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF

# Random123 kat_vectors, philox4x32 10 rounds: (counter c0..c3, key k0 k1) -> out
KAT = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF), (0xFFFFFFFF, 0xFFFFFFFF),
     (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def philox4x32_10(ctr, key):
    """ctr: [..., 4] uint32, key: [..., 2] uint32 (broadcast) -> [..., 4] uint32"""
    c = [np.asarray(ctr, np.uint64)[..., i] for i in range(4)]
    k0 = np.asarray(key, np.uint64)[..., 0] + np.zeros_like(c[0])
    k1 = np.asarray(key, np.uint64)[..., 1] + np.zeros_like(c[0])
    for r in range(10):
        if r:
            k0, k1 = (k0 + W0) & MASK, (k1 + W1) & MASK
        p0 = np.uint64(M0) * c[0]
        p1 = np.uint64(M1) * c[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & np.uint64(MASK)
        hi1, lo1 = p1 >> np.uint64(32), p1 & np.uint64(MASK)
        c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
    return np.stack(c, -1).astype(np.uint32)


def u01(x):
    """the device's 23-bit float in [0, 1): high 23 bits as the mantissa of [1, 2), minus 1"""
    bits = (np.asarray(x, np.uint32) >> np.uint32(9)) | np.uint32(0x3F800000)
    return bits.view(np.float32) - np.float32(1.0)


def uniforms5(seed, stream, ctr, rows):
    """[len(rows), 5] uniforms of mdp_device.h uniforms5 for counter (row, ctr, stream, 0|1)"""
    rows = np.asarray(rows, np.uint64)
    key = np.array([seed & MASK, (seed >> 32) & MASK], np.uint64)
    out = []
    for w in (0, 1):
        c = np.stack([rows, np.full_like(rows, ctr & MASK), np.full_like(rows, stream & MASK),
                      np.full_like(rows, w)], -1)
        out.append(philox4x32_10(c, key))
    a, b = out
    return u01(np.concatenate([a, b[:, :1]], 1))


def slot_uniforms(seed, stream, ctr, envs, count):
    """[len(envs), count] uniforms of mdp_kernels.hip env_reset_one: slot c is word
    c % 4 of the block at counter (env, ctr, stream, c / 4)"""
    envs = np.asarray(envs, np.uint64)
    key = np.array([seed & MASK, (seed >> 32) & MASK], np.uint64)
    blocks = []
    for q in range((count + 3) // 4):
        c = np.stack([envs, np.full_like(envs, ctr & MASK), np.full_like(envs, stream & MASK),
                      np.full_like(envs, q)], -1)
        blocks.append(philox4x32_10(c, key))
    return u01(np.concatenate(blocks, 1)[:, :count])


class ResetStream:
    """an `rng` for oracle/mpe.py's Scenario.reset(rng, E) that serves the
    device's reset uniforms: uniform() takes the next two slots per env in
    call order (entity order), integers() the slot after every position (the
    adversary goal, (int)(u * L) on the device)"""

    def __init__(self, u, n_entities):
        self.u, self.c, self.goal_slot = u, 0, 2 * n_entities

    def uniform(self, lo, hi, size):
        E, two = size
        assert two == 2
        lo32, span = np.float32(lo), np.float32(hi) - np.float32(lo)
        out = lo32 + span * self.u[:, self.c:self.c + 2]
        self.c += 2
        return out.astype(np.float64)

    def integers(self, lo, hi, size):
        g = (self.u[:, self.goal_slot] * np.float32(hi - lo)).astype(np.int64)
        return lo + np.minimum(g, hi - lo - 1)
