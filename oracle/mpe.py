"""Batched numpy fp64 restatement of the MPE scenarios (test oracle).

MPE (openai/multiagent-particle-envs, module ``multiagent``) is a third-party
dependency that is NOT vendored in the reference and NOT present in this
container; its version is unpinned by the reference (``README.md:23``).  Its
call sites in the reference are ``experiments/train.py:49-61`` (construction),
``:83`` (observation shapes), ``:104,128`` (reset), ``:114`` (step).  This is a
restatement of its published source (``multiagent/core.py`` World.step,
``multiagent/environment.py`` MultiAgentEnv.step/_set_action, and the
``simple``, ``simple_spread``, ``simple_adversary``, ``simple_tag`` scenarios).
Parity: UNPINNED (no fixture in the reference covers MPE).

State is batched over E env copies: ``pos[E, Ne, 2]``, ``vel[E, Ne, 2]``
(entities = agents then landmarks), plus ``goal[E]`` for simple_adversary.
"""
import numpy as np

DT = 0.1
DAMPING = 0.25
CONTACT_FORCE = 1e2
CONTACT_MARGIN = 1e-3


class Scenario:
    name = ""
    collaborative = False

    def __init__(self):
        self.n_agents = 0
        self.n_landmarks = 0
        self.size = []          # per entity
        self.collide = []
        self.movable = []
        self.accel = []         # per agent (None -> 5.0)
        self.max_speed = []     # per entity (None)
        self.adversary = []     # per agent

    @property
    def n_entities(self):
        return self.n_agents + self.n_landmarks

    def obs_dims(self):
        st = self.reset(np.random.default_rng(0), 1)
        return [o.shape[1] for o in self.observation(st)]

    # -- core.py World.step (apply_action_force, apply_environment_force,
    #    integrate_state); environment.py _set_action for Discrete spaces.
    def step(self, st, actions):
        """actions: [E, n_agents, 5] relaxed one-hot. Returns new state, obs_n, rew[E,N]."""
        pos = st["pos"].copy()
        vel = st["vel"].copy()
        E = pos.shape[0]
        ne = self.n_entities
        force = [None] * ne
        for i in range(self.n_agents):
            a = actions[:, i, :].astype(np.float64)
            u = np.zeros((E, 2))
            u[:, 0] += a[:, 1] - a[:, 2]
            u[:, 1] += a[:, 3] - a[:, 4]
            sens = 5.0 if self.accel[i] is None else self.accel[i]
            force[i] = u * sens
        for a in range(ne):
            for b in range(a + 1, ne):
                if not (self.collide[a] and self.collide[b]):
                    continue
                delta = pos[:, a] - pos[:, b]
                dist = np.sqrt(np.sum(np.square(delta), axis=1))
                dmin = self.size[a] + self.size[b]
                k = CONTACT_MARGIN
                pen = np.logaddexp(0, -(dist - dmin) / k) * k
                f = CONTACT_FORCE * delta / dist[:, None] * pen[:, None]
                if self.movable[a]:
                    force[a] = f if force[a] is None else f + force[a]
                if self.movable[b]:
                    force[b] = -f if force[b] is None else -f + force[b]
        for e in range(ne):
            if not self.movable[e]:
                continue
            v = vel[:, e] * (1 - DAMPING)
            if force[e] is not None:
                v = v + (force[e] / 1.0) * DT
            ms = self.max_speed[e]
            if ms is not None:
                sp = np.sqrt(np.square(v[:, 0]) + np.square(v[:, 1]))
                over = sp > ms
                scaled = v / np.sqrt(np.square(v[:, 0]) + np.square(v[:, 1]))[:, None] * ms
                v = np.where(over[:, None], scaled, v)
            vel[:, e] = v
            pos[:, e] = pos[:, e] + v * DT
        nst = dict(st)
        nst["pos"], nst["vel"] = pos, vel
        obs = self.observation(nst)
        rew = self.reward(nst)
        if self.collaborative:
            rew = np.repeat(rew.sum(1, keepdims=True), self.n_agents, axis=1)
        return nst, obs, rew

    @staticmethod
    def _dist(p, q):
        return np.sqrt(np.sum(np.square(p - q), axis=-1))

    def is_collision(self, st, i, j):
        d = self._dist(st["pos"][:, i], st["pos"][:, j])
        return d < (self.size[i] + self.size[j])

    def benchmark_data(self, st):
        """scenario.benchmark_data(agent, world) of every agent of the
        post-physics state (environment._get_info, train.py:57-60,139-141):
        a list over agents of per-env records [E, width]."""
        raise AttributeError(f"scenario {self.name!r} has no benchmark_data")

    def record(self, v, i):
        """the Python value MPE's benchmark_data returns for agent i (tuple / int /
        float) from its record row v (float array, MDP_BENCH_W wide)."""
        raise AttributeError(f"scenario {self.name!r} has no benchmark_data")


class Simple(Scenario):
    """scenarios/simple.py"""
    name = "simple"

    def __init__(self):
        super().__init__()
        self.n_agents, self.n_landmarks = 1, 1
        self.size = [0.05, 0.05]
        self.collide = [False, False]
        self.movable = [True, False]
        self.accel = [None]
        self.max_speed = [None, None]
        self.adversary = [False]

    def reset(self, rng, E):
        pos = np.zeros((E, 2, 2))
        pos[:, 0] = rng.uniform(-1, 1, (E, 2))
        pos[:, 1] = rng.uniform(-1, 1, (E, 2))
        return {"pos": pos, "vel": np.zeros((E, 2, 2))}

    def observation(self, st):
        p, v = st["pos"], st["vel"]
        return [np.concatenate([v[:, 0], p[:, 1] - p[:, 0]], 1)]

    def reward(self, st):
        p = st["pos"]
        return -np.sum(np.square(p[:, 0] - p[:, 1]), axis=1)[:, None]


class SimpleSpread(Scenario):
    """scenarios/simple_spread.py (3 agents, 3 landmarks, collaborative)."""
    name = "simple_spread"
    collaborative = True

    def __init__(self, n=3):
        super().__init__()
        self.n_agents, self.n_landmarks = n, n
        self.size = [0.15] * n + [0.05] * n
        self.collide = [True] * n + [False] * n
        self.movable = [True] * n + [False] * n
        self.accel = [None] * n
        self.max_speed = [None] * (2 * n)
        self.adversary = [False] * n

    def reset(self, rng, E):
        n = self.n_agents
        pos = np.zeros((E, 2 * n, 2))
        for i in range(n):
            pos[:, i] = rng.uniform(-1, 1, (E, 2))
        for i in range(n):
            pos[:, n + i] = 0.8 * rng.uniform(-1, 1, (E, 2))
        return {"pos": pos, "vel": np.zeros((E, 2 * n, 2))}

    def observation(self, st):
        n = self.n_agents
        p, v = st["pos"], st["vel"]
        out = []
        for i in range(n):
            parts = [v[:, i], p[:, i]]
            parts += [p[:, n + l] - p[:, i] for l in range(n)]
            parts += [p[:, j] - p[:, i] for j in range(n) if j != i]
            parts += [np.zeros((p.shape[0], 2)) for j in range(n) if j != i]   # other.state.c (silent)
            out.append(np.concatenate(parts, 1))
        return out

    def reward(self, st):
        n = self.n_agents
        p = st["pos"]
        base = np.zeros(p.shape[0])
        for l in range(n):
            d = np.stack([self._dist(p[:, a], p[:, n + l]) for a in range(n)], 1)
            base -= d.min(1)
        rew = np.zeros((p.shape[0], n))
        for i in range(n):
            r = base.copy()
            for a in range(n):                      # includes self (always a collision)
                r -= self.is_collision(st, a, i).astype(np.float64)
            rew[:, i] = r
        return rew

    def benchmark_data(self, st):
        """simple_spread.benchmark_data: (rew, collisions, min_dists, occupied_landmarks)."""
        n = self.n_agents
        p = st["pos"]
        E = p.shape[0]
        min_dists = np.zeros(E)
        occupied = np.zeros(E)
        for l in range(n):
            m = np.stack([self._dist(p[:, a], p[:, n + l]) for a in range(n)], 1).min(1)
            min_dists += m
            occupied += (m < 0.1)
        out = []
        for i in range(n):
            coll = np.zeros(E)
            for a in range(n):                      # is_collision(a, agent) incl. self
                coll += self.is_collision(st, a, i)
            out.append(np.stack([-min_dists - coll, coll, min_dists, occupied], 1))
        return out

    def record(self, v, i):
        return (float(v[0]), int(round(v[1])), float(v[2]), int(round(v[3])))


class SimpleAdversary(Scenario):
    """scenarios/simple_adversary.py (1 adversary + 2 good, 2 landmarks)."""
    name = "simple_adversary"

    def __init__(self, n_good=2, n_adv=1):
        super().__init__()
        n = n_good + n_adv
        self.n_agents, self.n_landmarks = n, n - 1
        self.size = [0.15] * n + [0.08] * (n - 1)
        self.collide = [False] * (2 * n - 1)
        self.movable = [True] * n + [False] * (n - 1)
        self.accel = [None] * n
        self.max_speed = [None] * (2 * n - 1)
        self.adversary = [i < n_adv for i in range(n)]

    def reset(self, rng, E):
        n, L = self.n_agents, self.n_landmarks
        goal = rng.integers(0, L, size=E)
        pos = np.zeros((E, n + L, 2))
        for i in range(n):
            pos[:, i] = rng.uniform(-1, 1, (E, 2))
        for l in range(L):
            pos[:, n + l] = 0.8 * rng.uniform(-1, 1, (E, 2))
        return {"pos": pos, "vel": np.zeros((E, n + L, 2)), "goal": goal}

    def _goal_pos(self, st):
        E = st["pos"].shape[0]
        return st["pos"][np.arange(E), self.n_agents + st["goal"]]

    def observation(self, st):
        n, L = self.n_agents, self.n_landmarks
        p = st["pos"]
        g = self._goal_pos(st)
        out = []
        for i in range(n):
            ent = [p[:, n + l] - p[:, i] for l in range(L)]
            oth = [p[:, j] - p[:, i] for j in range(n) if j != i]
            if self.adversary[i]:
                out.append(np.concatenate(ent + oth, 1))
            else:
                out.append(np.concatenate([g - p[:, i]] + ent + oth, 1))
        return out

    def reward(self, st):
        n = self.n_agents
        p = st["pos"]
        g = self._goal_pos(st)
        advs = [i for i in range(n) if self.adversary[i]]
        good = [i for i in range(n) if not self.adversary[i]]
        adv_rew = sum(self._dist(p[:, a], g) for a in advs)
        pos_rew = -np.min(np.stack([self._dist(p[:, a], g) for a in good], 1), axis=1)
        rew = np.zeros((p.shape[0], n))
        for i in range(n):
            if self.adversary[i]:
                rew[:, i] = -np.sum(np.square(p[:, i] - g), axis=1)
            else:
                rew[:, i] = pos_rew + adv_rew
        return rew

    def benchmark_data(self, st):
        """simple_adversary.benchmark_data: adversary |pos-goal|^2; good agents
        (|pos-lm_l|^2 for every landmark, |pos-goal|^2)."""
        n, L = self.n_agents, self.n_landmarks
        p = st["pos"]
        g = self._goal_pos(st)
        out = []
        for i in range(n):
            if self.adversary[i]:
                out.append(np.sum(np.square(p[:, i] - g), axis=1)[:, None])
            else:
                d = [np.sum(np.square(p[:, i] - p[:, n + l]), axis=1) for l in range(L)]
                d.append(np.sum(np.square(p[:, i] - g), axis=1))
                out.append(np.stack(d, 1))
        return out

    def record(self, v, i):
        if self.adversary[i]:
            return float(v[0])
        return tuple(float(x) for x in v[:self.n_landmarks + 1])


class SimpleTag(Scenario):
    """scenarios/simple_tag.py (default 3 adversaries + 1 good, 2 landmarks)."""
    name = "simple_tag"

    def __init__(self, n_adv=3, n_good=1, n_landmarks=2):
        super().__init__()
        n = n_adv + n_good
        self.n_agents, self.n_landmarks = n, n_landmarks
        self.adversary = [i < n_adv for i in range(n)]
        self.size = [0.075 if a else 0.05 for a in self.adversary] + [0.2] * n_landmarks
        self.collide = [True] * (n + n_landmarks)
        self.movable = [True] * n + [False] * n_landmarks
        self.accel = [3.0 if a else 4.0 for a in self.adversary]
        self.max_speed = [1.0 if a else 1.3 for a in self.adversary] + [None] * n_landmarks

    def reset(self, rng, E):
        n, L = self.n_agents, self.n_landmarks
        pos = np.zeros((E, n + L, 2))
        for i in range(n):
            pos[:, i] = rng.uniform(-1, 1, (E, 2))
        for l in range(L):
            pos[:, n + l] = rng.uniform(-0.9, 0.9, (E, 2))
        return {"pos": pos, "vel": np.zeros((E, n + L, 2))}

    def observation(self, st):
        n, L = self.n_agents, self.n_landmarks
        p, v = st["pos"], st["vel"]
        out = []
        for i in range(n):
            parts = [v[:, i], p[:, i]]
            parts += [p[:, n + l] - p[:, i] for l in range(L)]
            parts += [p[:, j] - p[:, i] for j in range(n) if j != i]
            parts += [v[:, j] for j in range(n) if j != i and not self.adversary[j]]
            out.append(np.concatenate(parts, 1))
        return out

    def reward(self, st):
        n = self.n_agents
        p = st["pos"]
        advs = [i for i in range(n) if self.adversary[i]]
        good = [i for i in range(n) if not self.adversary[i]]
        E = p.shape[0]
        rew = np.zeros((E, n))
        caught = np.zeros(E)
        for ag in good:
            for adv in advs:
                caught += self.is_collision(st, ag, adv)
        for i in range(n):
            if self.adversary[i]:
                rew[:, i] = 10.0 * caught
            else:
                r = np.zeros(E)
                for a in advs:
                    r -= 10.0 * self.is_collision(st, a, i)
                for d in range(2):
                    x = np.abs(p[:, i, d])
                    b = np.where(x < 0.9, 0.0,
                                 np.where(x < 1.0, (x - 0.9) * 10,
                                          np.minimum(np.exp(2 * x - 2), 10)))
                    r -= b
                rew[:, i] = r
        return rew

    def benchmark_data(self, st):
        """simple_tag.benchmark_data: adversary -> good agents in contact; good -> 0."""
        n = self.n_agents
        E = st["pos"].shape[0]
        out = []
        for i in range(n):
            c = np.zeros(E)
            if self.adversary[i]:
                for a in range(n):
                    if not self.adversary[a]:
                        c += self.is_collision(st, a, i)
            out.append(c[:, None])
        return out

    def record(self, v, i):
        return int(round(v[0]))


def make(name, **kw):
    return {"simple": Simple, "simple_spread": SimpleSpread,
            "simple_adversary": SimpleAdversary, "simple_tag": SimpleTag}[name](**kw)
