"""``MADDPGAgentTrainer`` drop-in (``maddpg/trainer/maddpg.py:112-196``).

Same constructor, methods, attributes and return values.  Every trainer built
in one session shares one device engine (see ``common/tf_util.py``); its
``update`` runs on the GPU in the reference's order: gates (``:162-165``),
``make_index`` from the global ``random`` stream (``:167``), gather of every
agent's buffer with that index (``:173-178``, fused into the grad kernels),
target actors + target critic + fp64 TD target (``:180-187``), critic step
(``:188``), actor step against the updated critic (``:191``), Polyak actor
then critic (``:193-194``).  ``update`` returns the 6 stats of ``:196`` as
the reference does: a ``list`` of numpy scalars with its dtypes (``q_loss``,
``p_loss`` and ``mean(target_q_next)`` fp32, the rest float64 --
``engine.UPDATE_STAT_DTYPES``), read after the update (the reference's
``session.run`` is synchronous too).

``model`` must be the reference's ``mlp_model`` (``train.py:39-46``: two
hidden ReLU layers of ``args.num_units`` and a linear output, TF
``fully_connected`` with Xavier-uniform weights) -- the architecture the HIP
kernels implement, for any ``--num-units`` up to 256.  It is recognised by name
(the reference's own function, or :func:`mlp_model` below), ``None`` selects
it; any other callable raises ``NotImplementedError`` rather than silently
training a different network.
"""
import numpy as np
import torch

from .. import AgentTrainer
from ..common import tf_util as U
from ..engine import update_stats
from .replay_buffer import ReplayBuffer


MAX_UNITS = 256


def mlp_model(input, num_outputs, scope, reuse=False, num_units=64, rnn_cell=None):
    """The reference's model function (``experiments/train.py:39-46``), kept as
    the architecture marker: the network itself is built by the device engine."""
    raise NotImplementedError("mlp_model is realised by the MI355X kernels; pass it to MADDPGAgentTrainer")


def check_model(model, num_units):
    """``model`` must describe the reference's mlp_model (see module doc)."""
    if model is not None and getattr(model, "__name__", None) != "mlp_model":
        raise NotImplementedError(
            f"model {model!r} is not mlp_model: the MI355X kernels implement the reference's 2-hidden-layer "
            "ReLU MLP (experiments/train.py:39-46) only")
    if not 1 <= int(num_units) <= MAX_UNITS:
        raise ValueError(f"--num-units {num_units}: the kernels take 1..{MAX_UNITS} hidden units")


class MADDPGAgentTrainer(AgentTrainer):
    def __init__(self, name, model, obs_shape_n, act_space_n, agent_index, args, local_q_func=False):
        self.name = name
        self.n = len(obs_shape_n)
        self.agent_index = agent_index
        self.args = args
        self.obs_shape_n = [tuple(s) for s in obs_shape_n]
        self.act_space_n = act_space_n
        self.local_q_func = local_q_func
        check_model(model, args.num_units)
        for sp in act_space_n:
            if getattr(sp, "n", 5) != 5:
                raise NotImplementedError("only Discrete(5) MPE action spaces are supported")
        self.session = U.get_session()
        self.session.register(self)
        self.replay_buffer = ReplayBuffer(1e6, _session=self.session, _agent=agent_index)
        self.max_replay_buffer_len = args.batch_size * args.max_episode_len
        self.replay_sample_index = None
        i = agent_index
        self.p_debug = {"p_values": lambda obs: self._eng().actor_logits(i, self._t(obs)).cpu().numpy(),
                        "target_act": lambda obs: self._eng().act(i, self._t(obs), target=True).cpu().numpy()}
        self.q_debug = {"q_values": lambda *a: self._q(a, False), "target_q_values": lambda *a: self._q(a, True)}

    # ------------------------------------------------------------ helpers
    def _eng(self):
        return self.session.engine()

    @staticmethod
    def _t(x):
        return torch.as_tensor(np.asarray(x, np.float32))

    def _q(self, arrays, target):
        n = self.n
        obs_n, act_n = list(arrays[:n]), list(arrays[n:2 * n])
        i = self.agent_index
        if self.local_q_func:                                          # maddpg.py:86-87
            x = np.concatenate([np.asarray(obs_n[i], np.float32), np.asarray(act_n[i], np.float32)], 1)
        else:                                                          # :85
            x = np.concatenate([np.asarray(a, np.float32) for a in obs_n + act_n], 1)
        return self._eng().q_values(i, self._t(x), target=target).cpu().numpy()

    # ------------------------------------------------------------ surface
    def action(self, obs):
        """act(obs[None])[0] (maddpg.py:151-152): actor + Gumbel-softmax sample."""
        return self._eng().act(self.agent_index, self._t(np.asarray(obs)[None])).cpu().numpy()[0]

    def experience(self, obs, act, rew, new_obs, done, terminal):
        self.replay_buffer.add(obs, act, rew, new_obs, float(done))    # :154-156

    def preupdate(self):
        self.replay_sample_index = None

    def update(self, agents, t):
        if len(self.replay_buffer) < self.max_replay_buffer_len:    # :162-163
            return None
        if not t % 100 == 0:                                          # :164-165
            return None
        for a in agents:
            if a.session is not self.session:
                raise RuntimeError("all agents of an update must share one session")
        eng = self._eng()
        self.session.flush()
        idx = self.replay_buffer.make_index_device(self.args.batch_size)   # :167
        self.replay_sample_index = idx
        eng.update(self.agent_index, idx=idx)                           # :173-194
        host, ev = eng.stats_future(self.agent_index)
        ev.synchronize()
        if self.session.check_nan:                                      # tf_util.py:366-368
            U.check_nan(eng)
        return update_stats(host.tolist())                              # :196
