"""``ReplayBuffer`` drop-in (``maddpg/trainer/replay_buffer.py:5-85``).

Same constructor and methods; the transitions live in the device replay ring
of a libmaddpg_hip engine instead of a Python list:

* ``add`` keeps the reference's ring bookkeeping (``_next_idx``, ``len``) on
  the host and stages rows, written to the device in one launch when a device
  read needs them (``k_put_agent``).
* ``make_index`` draws on the DEVICE MT19937 from the module-global
  ``random`` state and writes the advanced state back, so the indices and the
  global RNG stream are bit-identical to ``random.randint`` (``:46-47``).
* ``sample_index``/``sample``/``collect`` gather on the device
  (``k_gather_rows``) and return the reference's dtypes (obs/rew/done float64,
  act float32; values are stored as fp32).

A standalone buffer builds a private single-agent engine on the first
``add``; a trainer's buffer is a column view of the session's joint ring.
"""
import numpy as np
import torch

from ..common import tf_util as U

ACT = 5


class ReplayBuffer(object):
    def __init__(self, size, _session=None, _agent=0):
        self._maxsize = int(size)
        self._next_idx = 0
        self._len = 0
        self._session = _session
        self._agent = _agent
        self._engine = None
        self._pending = []          # (position, obs, act, rew, obs_tp1, done)
        if _session is not None:
            _session.register_buffer(self)

    # ------------------------------------------------------------ storage
    def _eng(self, obs_dim=None):
        if self._session is not None:
            return self._session.engine()
        if self._engine is None:
            if obs_dim is None:
                raise RuntimeError("empty standalone ReplayBuffer")
            from ..engine import Engine
            self._engine = Engine([obs_dim], batch_size=1, capacity=self._maxsize)
        return self._engine

    def __len__(self):
        return self._len

    def clear(self):
        self._pending = []
        self._len = 0
        self._next_idx = 0

    def add(self, obs_t, action, reward, obs_tp1, done):
        self._pending.append((self._next_idx, obs_t, action, reward, obs_tp1, done))
        if self._next_idx >= self._len:
            self._len += 1
        self._next_idx = (self._next_idx + 1) % self._maxsize

    def flush(self):
        if not self._pending:
            return
        obs0 = np.asarray(self._pending[0][1]).ravel()
        eng = self._eng(obs0.size)
        o = eng.obs_dims[self._agent]
        k = len(self._pending)
        cols = np.empty((k, 2 * o + ACT + 2), np.float32)
        pos = np.empty(k, np.int64)
        for r, (p, ob, a, rw, ob1, d) in enumerate(self._pending):
            pos[r] = p
            cols[r, :o] = np.asarray(ob, np.float32).ravel()
            cols[r, o:o + ACT] = np.asarray(a, np.float32).ravel()
            cols[r, o + ACT:2 * o + ACT] = np.asarray(ob1, np.float32).ravel()
            cols[r, 2 * o + ACT] = rw
            cols[r, 2 * o + ACT + 1] = d
        # later adds to the same position win (ring overwrite): keep the last one
        _, last = np.unique(pos[::-1], return_index=True)
        keep = np.sort(k - 1 - last)
        eng.put_agent(self._agent, torch.from_numpy(pos[keep]), torch.from_numpy(cols[keep]))
        self._pending = []

    # ------------------------------------------------------------ indices
    def make_index_device(self, batch_size):
        """device int32 indices drawn from (and advancing) the global ``random`` stream."""
        self.flush()
        eng = self._eng()
        if self._len == 0:
            raise ValueError("empty range for randrange() (replay buffer is empty)")
        eng.set_ring(self._len, self._next_idx % eng.capacity)
        st = U.sync_rng_to_device(eng)
        idx = eng.make_index(batch_size)
        U.sync_rng_from_device(eng, st)
        return idx

    def make_index(self, batch_size):
        return self.make_index_device(batch_size).cpu().tolist()

    def make_latest_index(self, batch_size):
        idx = [(self._next_idx - 1 - i) % self._maxsize for i in range(batch_size)]
        np.random.shuffle(idx)
        return idx

    # ------------------------------------------------------------- gather
    def sample_index(self, idxes):
        self.flush()
        eng = self._eng()
        if isinstance(idxes, torch.Tensor):
            idx = idxes.to(torch.int32)
        else:
            idx = torch.as_tensor(np.asarray(list(idxes), np.int64).astype(np.int32))
        rows = eng.sample_rows(idx).cpu().numpy()
        oo, ao, no, ro, do, _stride = eng.row_layout[self._agent]
        o = eng.obs_dims[self._agent]
        return (rows[:, oo:oo + o].astype(np.float64), rows[:, ao:ao + ACT].astype(np.float32),
                rows[:, ro].astype(np.float64), rows[:, no:no + o].astype(np.float64),
                rows[:, do].astype(np.float64))

    def sample(self, batch_size):
        if batch_size > 0:
            idxes = self.make_index(batch_size)
        else:
            idxes = range(0, self._len)
        return self.sample_index(idxes)

    def collect(self):
        return self.sample(-1)
