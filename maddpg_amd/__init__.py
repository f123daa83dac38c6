"""maddpg_amd -- MI355X-native MADDPG training hot path.

Drop-in for the reference's ``maddpg`` package surface on this path:
``AgentTrainer`` (maddpg/__init__.py:1-15), ``trainer.maddpg.MADDPGAgentTrainer``
and ``trainer.replay_buffer.ReplayBuffer``; the compute runs in
``libmaddpg_hip.so`` (hand-written HIP for gfx950) through ``_lib``.
"""


class AgentTrainer(object):
    """Abstract trainer surface (maddpg/__init__.py:1-15)."""

    def __init__(self, name, model, obs_shape, act_space, args):
        raise NotImplementedError()

    def action(self, obs):
        raise NotImplementedError()

    def process_experience(self, obs, act, rew, new_obs, done, terminal):
        raise NotImplementedError()

    def preupdate(self):
        raise NotImplementedError()

    def update(self, agents):
        raise NotImplementedError()
