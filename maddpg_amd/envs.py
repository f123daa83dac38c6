"""Scenario metadata for the device MPE environments.

Mirrors what ``experiments/train.py:48-61`` obtains from MPE's
``scenarios.load(name).Scenario().make_world()``: the number of policy agents
(``env.n``), per-agent observation widths (``env.observation_space[i].shape``,
``train.py:83``) and ``Discrete(5)`` action spaces (``train.py:69,73``).
The physics itself runs in ``k_rollout`` (maddpg_amd/csrc/mdp_kernels.hip).
"""
from dataclasses import dataclass, field
from typing import List

ACT_DIM = 5


class Discrete:
    """Minimal stand-in for ``gym.spaces.Discrete`` (gym is not installed)."""

    def __init__(self, n):
        self.n = int(n)

    def __repr__(self):
        return f"Discrete({self.n})"


@dataclass
class ScenarioSpec:
    name: str
    n_agents: int
    num_adversaries: int
    obs_dims: List[int] = field(default_factory=list)

    @property
    def action_space(self):
        return [Discrete(ACT_DIM) for _ in range(self.n_agents)]

    @property
    def observation_shapes(self):
        return [(o,) for o in self.obs_dims]


def spec(name, n_agents=None, num_adversaries=None):
    """Scenario table (upstream make_world defaults unless overridden)."""
    if name == "simple":
        return ScenarioSpec(name, 1, 0, [4])
    if name == "simple_spread":
        n = 3 if n_agents is None else n_agents
        return ScenarioSpec(name, n, 0, [4 + 2 * n + 4 * (n - 1)] * n)
    if name == "simple_adversary":
        n = 3 if n_agents is None else n_agents
        na = 1 if num_adversaries is None else num_adversaries
        dims = [(0 if i < na else 2) + 4 * (n - 1) for i in range(n)]
        return ScenarioSpec(name, n, na, dims)
    if name == "simple_tag":
        n = 4 if n_agents is None else n_agents
        na = 3 if num_adversaries is None else num_adversaries
        ng = n - na
        L = 2
        dims = [4 + 2 * L + 2 * (n - 1) + 2 * (ng if i < na else ng - 1) for i in range(n)]
        return ScenarioSpec(name, n, na, dims)
    raise ValueError(f"unknown scenario {name!r}")


def bench_record(sp, row, i):
    """Python value of agent i's scenario benchmark_data() (MPE returns tuples /
    ints / floats; train.py:141 stores them in info_n['n']) from its device
    record row (mdp_env_step_bench, MDP_BENCH_W floats)."""
    if sp.name == "simple_spread":
        return (float(row[0]), int(round(row[1])), float(row[2]), int(round(row[3])))
    if sp.name == "simple_adversary":
        if i < sp.num_adversaries:
            return float(row[0])
        return tuple(float(x) for x in row[:sp.n_agents])   # n-1 landmarks + goal
    if sp.name == "simple_tag":
        return int(round(row[0]))
    raise AttributeError(f"scenario {sp.name!r} has no benchmark_data")
