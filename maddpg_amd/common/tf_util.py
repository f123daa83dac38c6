"""Session plumbing of the drop-in surface (``maddpg/common/tf_util.py``).

The reference keeps all trainer state in the default TF session
(``get_session`` ``tf_util.py:189-191``, ``single_threaded_session``
``:202-204``, ``initialize`` ``:210-214``, ``save_state``/``load_state``
``:259-273``).  Here the equivalent is a :class:`Session`: the
``MADDPGAgentTrainer`` objects built under it register themselves, and the
first ``initialize()`` (or first compute call) builds ONE device engine for
all of them -- one joint replay buffer, one parameter arena -- because the
reference's update reads every agent's buffer with a shared index set
(``maddpg.py:167-178``).
"""
import contextlib
import os
import random

import numpy as np

_DEFAULT = None


class Session:
    def __init__(self, seed=None, check_nan=None):
        self.trainers = []
        self.buffers = []
        self._engine = None
        self.seed = seed
        # the reference's _Function(check_nan) (tf_util.py:322,366-368; off there):
        # when on, every update() checks the device state and raises "Nan detected"
        self.check_nan = (os.environ.get("MDP_CHECK_NAN", "0") == "1") if check_nan is None else bool(check_nan)

    # trainers and their replay buffers register here
    def register(self, trainer):
        if self._engine is not None:
            raise RuntimeError("cannot add trainers after the session was initialised")
        self.trainers.append(trainer)

    def register_buffer(self, buf):
        self.buffers.append(buf)

    @property
    def initialized(self):
        return self._engine is not None

    def engine(self):
        if self._engine is None:
            self.initialize()
        return self._engine

    def initialize(self):
        """U.initialize(): build the engine and initialise every variable (Xavier,
        targets independent of the online nets, Adam slots zero)."""
        if self._engine is not None:
            return self._engine
        if not self.trainers:
            raise RuntimeError("no MADDPGAgentTrainer registered in this session")
        from ..engine import Engine
        t0 = self.trainers[0]
        args = t0.args
        n = t0.n
        for t in self.trainers:
            if t.n != n:
                raise ValueError("trainers disagree on the number of agents")
        by_index = {t.agent_index: t for t in self.trainers}
        obs_dims = [int(np.prod(s)) for s in t0.obs_shape_n]
        local_q = [bool(by_index[i].local_q_func) if i in by_index else False for i in range(n)]
        seed = self.seed if self.seed is not None else int(getattr(args, "seed", 0) or 0)
        self._engine = Engine(obs_dims, local_q, num_units=args.num_units, batch_size=args.batch_size,
                              max_episode_len=args.max_episode_len, capacity=int(1e6), lr=args.lr,
                              gamma=args.gamma, seed=seed)
        self._engine.init_params(seed)
        return self._engine

    def flush(self):
        for b in self.buffers:
            b.flush()

    def close(self):
        if self._engine is not None:
            self._engine.close()
            self._engine = None


def get_session():
    """Recently made session (tf_util.get_session); a default one is created on demand."""
    global _DEFAULT
    if _DEFAULT is None:
        _DEFAULT = Session()
    return _DEFAULT


def make_session(num_cpu=1, seed=None, check_nan=None):
    """tf_util.make_session: num_cpu is accepted for signature parity (compute is on the GPU)."""
    global _DEFAULT
    _DEFAULT = Session(seed=seed, check_nan=check_nan)
    return _DEFAULT


@contextlib.contextmanager
def single_threaded_session(seed=None, check_nan=None):
    """``with U.single_threaded_session():`` (experiments/train.py:79)."""
    global _DEFAULT
    prev = _DEFAULT
    sess = make_session(1, seed, check_nan)
    try:
        yield sess
    finally:
        sess.close()
        _DEFAULT = prev


def initialize():
    """U.initialize() (tf_util.py:210-214)."""
    return get_session().initialize()


def save_state(fname, saver=None, fmt="npz"):
    """U.save_state (tf_util.py:267-273): every variable of every agent
    (fmt="tf1": a TF1 checkpoint with the reference's variable names)."""
    return get_session().engine().save_state(fname, fmt)


def load_state(fname, saver=None):
    """U.load_state (tf_util.py:259-264): a TF1 checkpoint at prefix fname
    (tf.train.Saver's files) or the .npz save_state writes."""
    return get_session().engine().load_state(fname)


def check_nan(engine):
    """tf_util.py:366-368 on the device state: raise RuntimeError("Nan detected")
    when any parameter, target, Adam slot or update stat is NaN or Inf"""
    if engine.check_finite():
        raise RuntimeError("Nan detected")


def sync_rng_to_device(engine):
    """Copy the module-global CPython RNG state into the device MT19937."""
    st = random.getstate()
    engine.set_rng_state(np.array(st[1], dtype=np.uint64))
    return st


def sync_rng_from_device(engine, st):
    """Write the device MT19937 state back into the module-global RNG."""
    new = engine.get_rng_state()
    random.setstate((st[0], tuple(int(x) for x in new), st[2]))
