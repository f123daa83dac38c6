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
    # (a float64 draw near 1 rounds to 1.0 in fp32, where -log(-log u) is infinite: capped below 1)
    top = np.nextafter(np.float32(1), np.float32(0))
    u_tgt = np.minimum(rng.uniform(1e-6, 1.0, size=(n, n, B, ACT)).astype(np.float32), top)
    u_act = np.minimum(rng.uniform(1e-6, 1.0, size=(n, B, ACT)).astype(np.float32), top)
    return dict(data=data, params=params, idx=idx, u_tgt=u_tgt, u_act=u_act, local_q=local_q)


def relu_margin_clean_idx(c, margin=1e-5, max_iter=20):
    """Replace, agent by agent, every batch position whose row puts a ReLU input of
    a net that agent's round-start update evaluates within `margin` x (that
    layer's largest |input| over the batch) of zero, by another random row.

    fp32 evaluates such an input with a rounding error of ~1e-7 of the layer's
    scale and in a summation order of its own, so the ReLU mask of that (row,
    unit) can come out either way in two correct fp32 implementations, and one
    flipped mask moves a sum over 4,096 rows by ~1e-4 of its largest entry.
    With no input that close to zero, the device and the restatement must agree
    to fp32 summation order.  Modifies c["idx"] in place (throughput-mode round:
    every net at its round-start value); returns the number of positions replaced.
    Nets checked for agent i: every target actor on obs' (sample u_tgt[i][j]),
    target critic i on [obs' | a~], critic i on the replay input and on the
    actor step's input (a_i := the sample of actor i with u_act[i]), actor i."""
    from oracle import nets
    data, params, n = c["data"], c["params"], len(c["params"])
    lq = c["local_q"]
    rng = np.random.default_rng(12345)
    L = data[0][0].shape[0]
    f64 = lambda p: {k: np.asarray(v, np.float64) for k, v in p.items()}  # noqa: E731

    def fwd(p, x):
        z1 = x @ p["W1"] + p["b1"]
        z2 = np.maximum(z1, 0) @ p["W2"] + p["b2"]
        return np.maximum(z2, 0) @ p["W3"] + p["b3"], (z1, z2)

    def gsm(logits, u):
        z = logits - np.log(-np.log(u.astype(np.float64)))
        e = np.exp(z - z.max(-1, keepdims=True))
        return e / e.sum(-1, keepdims=True)

    def bad(zs):
        out = np.zeros(zs[0].shape[0], bool)
        for z in zs:
            out |= (np.abs(z) < margin * np.abs(z).max()).any(1)
        return out

    P = [{w: f64(params[i][w]) for w in ("actor", "critic", "tgt_actor", "tgt_critic")} for i in range(n)]
    replaced = 0
    for i in range(n):
        for _ in range(max_iter):
            rows = c["idx"][i]
            obs = [np.asarray(data[j][0][rows], np.float64) for j in range(n)]
            act = [np.asarray(data[j][1][rows], np.float64) for j in range(n)]
            nobs = [np.asarray(data[j][3][rows], np.float64) for j in range(n)]
            zs = []
            at = []
            for j in range(n):
                lg, z = fwd(P[j]["tgt_actor"], nobs[j])
                zs += list(z)
                at.append(gsm(lg, c["u_tgt"][i][j]))
            xt = np.concatenate([nobs[i], at[i]], 1) if lq[i] else np.concatenate(nobs + at, 1)
            zs += list(fwd(P[i]["tgt_critic"], xt)[1])
            xc = np.concatenate([obs[i], act[i]], 1) if lq[i] else np.concatenate(obs + act, 1)
            zs += list(fwd(P[i]["critic"], xc)[1])
            lg, z = fwd(P[i]["actor"], obs[i])
            zs += list(z)
            a_in = list(act)
            a_in[i] = gsm(lg, c["u_act"][i])
            xp = np.concatenate([obs[i], a_in[i]], 1) if lq[i] else np.concatenate(obs + a_in, 1)
            zs += list(fwd(P[i]["critic"], xp)[1])
            b = bad(zs)
            if not b.any():
                break
            replaced += int(b.sum())
            c["idx"][i][b] = rng.integers(0, L, size=int(b.sum())).astype(np.int32)
        else:
            raise RuntimeError(f"agent {i}: no ReLU-margin-clean batch after {max_iter} resamplings")
    return replaced
