"""Restatement of CPython's Mersenne Twister and ``random.randint`` (test oracle).

The reference draws replay indices with the module-global CPython RNG:
``[random.randint(0, len(self._storage) - 1) for _ in range(batch_size)]``
(``maddpg/trainer/replay_buffer.py:46-47``).  CPython 3.10 implements that as

* ``Modules/_randommodule.c``: ``init_genrand``/``init_by_array`` seeding,
  ``genrand_uint32`` (MT19937 twist + tempering), ``getrandbits(k<=32)`` =
  ``genrand_uint32() >> (32 - k)``;
* ``Lib/random.py``: ``randint(a, b) = randrange(a, b+1)`` ->
  ``a + _randbelow(n)``; ``_randbelow_with_getrandbits(n)``: ``k =
  n.bit_length(); r = getrandbits(k); while r >= n: r = getrandbits(k)``.

State layout is CPython's: 624 words + the read position ``pos`` (0..624),
exactly ``random.getstate()[1]``.
"""
import numpy as np

N = 624
M = 397
MATRIX_A = 0x9908B0DF
UPPER = 0x80000000
LOWER = 0x7FFFFFFF
MASK32 = 0xFFFFFFFF


def init_genrand(s):
    mt = [0] * N
    mt[0] = s & MASK32
    for i in range(1, N):
        mt[i] = (1812433253 * (mt[i - 1] ^ (mt[i - 1] >> 30)) + i) & MASK32
    return mt


def init_by_array(key):
    """_randommodule.c init_by_array."""
    mt = init_genrand(19650218)
    i, j = 1, 0
    klen = len(key)
    for _ in range(max(N, klen)):
        mt[i] = ((mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525)) + key[j] + j) & MASK32
        i += 1
        j += 1
        if i >= N:
            mt[0] = mt[N - 1]
            i = 1
        if j >= klen:
            j = 0
    for _ in range(N - 1):
        mt[i] = ((mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941)) - i) & MASK32
        i += 1
        if i >= N:
            mt[0] = mt[N - 1]
            i = 1
    mt[0] = 0x80000000
    return mt


def seed_key(seed):
    """random.seed(int): key = little-endian 32-bit words of abs(seed)."""
    n = abs(int(seed))
    key = []
    while n:
        key.append(n & MASK32)
        n >>= 32
    return key or [0]


def twist(mt):
    """One MT19937 generation step over all 624 words (sequential reference)."""
    mt = list(mt)
    for kk in range(N):
        y = (mt[kk] & UPPER) | (mt[(kk + 1) % N] & LOWER)
        mt[kk] = mt[(kk + M) % N] ^ (y >> 1) ^ (MATRIX_A if (y & 1) else 0)
    return mt


def temper(y):
    y ^= y >> 11
    y ^= (y << 7) & 0x9D2C5680
    y ^= (y << 15) & 0xEFC60000
    y ^= y >> 18
    return y & MASK32


class MT19937:
    """CPython-compatible generator; ``state()`` matches ``random.getstate()[1]``."""

    def __init__(self, seed=None, state=None):
        if state is not None:
            self.mt = [int(x) & MASK32 for x in state[:N]]
            self.pos = int(state[N])
        else:
            self.mt = init_by_array(seed_key(0 if seed is None else seed))
            self.pos = N

    def state(self):
        return tuple(self.mt) + (self.pos,)

    def genrand_uint32(self):
        if self.pos >= N:
            self.mt = twist(self.mt)
            self.pos = 0
        y = self.mt[self.pos]
        self.pos += 1
        return temper(y)

    def getrandbits(self, k):
        assert 0 < k <= 32
        return self.genrand_uint32() >> (32 - k)

    def randbelow(self, n):
        if n <= 0:
            return 0
        k = int(n).bit_length()
        r = self.getrandbits(k)
        while r >= n:
            r = self.getrandbits(k)
        return r

    def randint(self, a, b):
        return a + self.randbelow(b - a + 1)

    def make_index(self, length, batch_size):
        """replay_buffer.py:46-47 on this generator."""
        return np.array([self.randint(0, length - 1) for _ in range(batch_size)], dtype=np.int64)
