"""Generate the replay-buffer golden fixtures by running the REFERENCE itself.

Run in the build container only (the reference never travels):

    python tests/golden/make_golden.py

It imports ``ReplayBuffer`` from ``/root/reference/maddpg/trainer/replay_buffer.py``
(pure Python + numpy; no TensorFlow needed), seeds the module-global CPython
RNG exactly as a user of ``experiments/train.py`` would (``random.seed``),
fills one buffer per agent through ``add`` (``replay_buffer.py:25-32``), then
replays the per-round call sequence of ``maddpg/trainer/maddpg.py:167-178``:
agent i draws ``make_index(B)`` from its own buffer (agent 0 first) and every
agent's buffer is gathered with that index via ``sample_index``.

Stored per case (``replay_golden.npz``):
* ``idx``   int32 [N, B]   -- the reference's indices, agent-major;
* ``state`` uint32 [625]   -- ``random.getstate()[1]`` after the draws;
* ``gather_sha256``        -- sha256 over every array ``sample_index`` returned
  (in the reference's dtypes: obs/rew/done float64, act float32);
* small cases also keep the gathered arrays themselves.
The buffer contents are regenerated bit-identically by ``make_data`` (seeded
numpy), so only the index stream and the digests need to be stored.
"""
import hashlib
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ACT = 5

# (name, rng_seed, capacity, n_added, batch, obs_dims)
CASES = []
for s in (0, 1, 12345):
    CASES += [
        (f"spread_s{s}", s, 1_000_000, 25_600, 1024, (18, 18, 18)),
        (f"simple_s{s}", s, 1_000_000, 25_600, 1024, (4,)),
        (f"wrap_s{s}", s, 1000, 2500, 1024, (8, 10, 10)),
        (f"tag6_s{s}", s, 1_000_000, 51_200, 4096, (22, 22, 22, 22, 20, 20)),
        (f"small_s{s}", s, 64, 100, 64, (18, 18, 18)),
    ]
FULL_GATHER = lambda name: name.startswith("small")


def make_data(case_seed, n_added, obs_dims):
    """Per-agent transition streams (added in order 0..n_added-1).

    Values are float32-representable so a float32 device buffer holds them
    exactly; obs/rew/done are float64 like MPE's outputs, act float32 like
    the actor's output (maddpg.py:151-156)."""
    rng = np.random.default_rng(10_000 + case_seed)
    out = []
    for o in obs_dims:
        obs = rng.uniform(-1, 1, (n_added, o)).astype(np.float32).astype(np.float64)
        z = rng.normal(size=(n_added, ACT)).astype(np.float32)
        e = np.exp(z - z.max(1, keepdims=True))
        act = (e / e.sum(1, keepdims=True)).astype(np.float32)
        rew = rng.normal(-3, 1, n_added).astype(np.float32).astype(np.float64)
        obs_next = rng.uniform(-1, 1, (n_added, o)).astype(np.float32).astype(np.float64)
        done = (rng.random(n_added) < 0.02).astype(np.float64)
        out.append((obs, act, rew, obs_next, done))
    return out


def digest(arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def main():
    sys.path.insert(0, "/root/reference")
    from maddpg.trainer.replay_buffer import ReplayBuffer   # the reference, run as-is

    store = {}
    for ci, (name, seed, cap, n_added, B, dims) in enumerate(CASES):
        data = make_data(ci, n_added, dims)
        bufs = []
        for (obs, act, rew, obs_next, done) in data:
            rb = ReplayBuffer(cap)
            for r in range(n_added):
                rb.add(obs[r], act[r], float(rew[r]), obs_next[r], float(done[r]))
            bufs.append(rb)
        random.seed(seed)
        idx = []
        gathered = []
        for i in range(len(dims)):                            # maddpg.py:167-178
            ix = bufs[i].make_index(B)
            idx.append(ix)
            per_agent = [bufs[j].sample_index(ix) for j in range(len(dims))]
            own = bufs[i].sample_index(ix)
            arrs = []
            for (o, a, _r, on, _d) in per_agent:
                arrs += [o, a, on]
            arrs += [own[2], own[4]]
            gathered.append(arrs)
        state = np.array(random.getstate()[1], dtype=np.uint64).astype(np.uint32)
        store[f"{name}/idx"] = np.array(idx, dtype=np.int32)
        store[f"{name}/state"] = state
        store[f"{name}/meta"] = np.array([ci, seed, cap, n_added, B] + list(dims), dtype=np.int64)
        store[f"{name}/gather_sha256"] = np.array(
            [digest(g) for g in gathered])
        if FULL_GATHER(name):
            for i, g in enumerate(gathered):
                for k, a in enumerate(g):
                    store[f"{name}/g{i}_{k}"] = a
        print(name, "done", store[f"{name}/idx"].shape)
    np.savez_compressed(os.path.join(HERE, "replay_golden.npz"), **store)


if __name__ == "__main__":
    main()
