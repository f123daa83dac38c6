"""Restatement of ``maddpg/trainer/replay_buffer.py`` (test oracle).

Per-agent ring buffer of transitions; ``make_index`` draws from a CPython-
compatible MT19937 (``oracle.pyrandom``) standing in for the module-global
``random`` used by the reference (``replay_buffer.py:46-47``).
"""
import numpy as np

from .pyrandom import MT19937


class ReplayBuffer:
    def __init__(self, size):                       # replay_buffer.py:6-16
        self._storage = []
        self._maxsize = int(size)
        self._next_idx = 0

    def __len__(self):                              # :18-19
        return len(self._storage)

    def add(self, obs_t, action, reward, obs_tp1, done):   # :25-32
        data = (obs_t, action, reward, obs_tp1, done)
        if self._next_idx >= len(self._storage):
            self._storage.append(data)
        else:
            self._storage[self._next_idx] = data
        self._next_idx = (self._next_idx + 1) % self._maxsize

    def _encode_sample(self, idxes):                # :34-44
        obses_t, actions, rewards, obses_tp1, dones = [], [], [], [], []
        for i in idxes:
            obs_t, action, reward, obs_tp1, done = self._storage[i]
            obses_t.append(np.asarray(obs_t))
            actions.append(np.asarray(action))
            rewards.append(reward)
            obses_tp1.append(np.asarray(obs_tp1))
            dones.append(done)
        return (np.array(obses_t), np.array(actions), np.array(rewards),
                np.array(obses_tp1), np.array(dones))

    def make_index(self, batch_size, rng: MT19937):  # :46-47
        return rng.make_index(len(self._storage), batch_size)

    def sample_index(self, idxes):                  # :55-56
        return self._encode_sample(idxes)
