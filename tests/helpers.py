"""Shared builders for the parity tests (host side only)."""
import numpy as np

from tests.golden.make_golden import ACT, make_data


def row_layout(dims):
    """Joint replay row layout (maddpg_amd/csrc/mdp_topo.h)."""
    n, S = len(dims), int(sum(dims))
    offs = np.concatenate([[0], np.cumsum(dims)]).astype(int)
    lay = []
    for j in range(n):
        lay.append(dict(obs=offs[j], act=S + ACT * j, nobs=S + ACT * n + offs[j],
                        rew=2 * S + ACT * n + j, done=2 * S + ACT * n + n + j))
    stride = (2 * S + (ACT + 2) * n + 3) // 4 * 4
    return lay, stride


def joint_rows(data, dims):
    """data[j] = (obs, act, rew, obs_next, done) streams -> [L, stride] float32 rows."""
    lay, stride = row_layout(dims)
    L = data[0][0].shape[0]
    rows = np.zeros((L, stride), np.float32)
    for j, (o, a, r, on, d) in enumerate(data):
        lj = lay[j]
        rows[:, lj["obs"]:lj["obs"] + dims[j]] = o
        rows[:, lj["act"]:lj["act"] + ACT] = a
        rows[:, lj["nobs"]:lj["nobs"] + dims[j]] = on
        rows[:, lj["rew"]] = r
        rows[:, lj["done"]] = d
    return rows


def ring_storage(data, cap):
    """Contents of the reference ring after adding all rows in order (replay_buffer.py:25-32)."""
    L = data[0][0].shape[0]
    n = min(L, cap)
    src = np.empty(n, np.int64)
    for a in range(L):
        src[a % cap] = a
    return [tuple(x[src] for x in d) for d in data]


def golden_case(golden, name):
    meta = golden[f"{name}/meta"]
    ci, seed, cap, n_added, B = (int(x) for x in meta[:5])
    dims = [int(x) for x in meta[5:]]
    return dict(name=name, ci=ci, seed=seed, cap=cap, n_added=n_added, B=B, dims=dims,
                idx=golden[f"{name}/idx"], state=golden[f"{name}/state"],
                sha=[str(s) for s in golden[f"{name}/gather_sha256"]],
                data=lambda: make_data(ci, n_added, dims))


def case_names(golden):
    return sorted({k.split("/")[0] for k in golden.files})


def synthetic_trainer_case(dims, B, L, seed, local_q=None, H=64):
    """Replay contents, weights of all four nets per agent and injected noise."""
    from oracle import nets
    rng = np.random.default_rng(seed)
    data = make_data(seed + 77, L, dims)
    n = len(dims)
    S = sum(dims)
    local_q = [False] * n if local_q is None else local_q
    params = []
    for i in range(n):
        cin = dims[i] + ACT if local_q[i] else S + ACT * n
        params.append(dict(actor=nets.xavier_init(rng, dims[i], ACT, H),
                           critic=nets.xavier_init(rng, cin, 1, H),
                           tgt_actor=nets.xavier_init(rng, dims[i], ACT, H),
                           tgt_critic=nets.xavier_init(rng, cin, 1, H)))
    idx = rng.integers(0, L, size=(n, B)).astype(np.int32)
    u_tgt = rng.uniform(1e-6, 1.0, size=(n, n, B, ACT)).astype(np.float32)
    u_act = rng.uniform(1e-6, 1.0, size=(n, B, ACT)).astype(np.float32)
    return dict(data=data, params=params, idx=idx, u_tgt=u_tgt, u_act=u_act, local_q=local_q)
