"""Engine: one libmaddpg_hip handle + its device arena (PyTorch storage only).

Everything the reference keeps in the TF session (weights, targets, Adam
slots, beta powers -- ``tf_util.py:189-214``) and in the per-agent Python
replay lists (``replay_buffer.py``) lives in one device arena owned by a
``torch.uint8`` CUDA tensor; all compute is launched by the HIP library on
the engine's stream.  No CPU fallback exists: construction raises without a
GPU or without the built library.
"""
import ctypes
import os

import numpy as np
import torch

from . import _lib
from ._lib import MdpConfig, MdpTensorInfo

TENSOR_NAMES = ("W1", "b1", "W2", "b2", "W3", "b3")

# the dtypes of update()'s return value in the reference (maddpg.py:196):
# q_loss, p_loss are the fp32 scalars U.function fetches from TF1 (:91, :54-56);
# np.mean(target_q_next) is the mean of an fp32 array (fp32, :185); the mean
# and std of the fp64 TD target and the mean reward are float64 (:186)
UPDATE_STAT_DTYPES = (np.float32, np.float32, np.float64, np.float64, np.float32, np.float64)


def update_stats(vals):
    """the 6 device stats (fp64, mdp_get_stats) as the reference's list of numpy scalars"""
    return [dt(v) for dt, v in zip(UPDATE_STAT_DTYPES, list(vals))]


class Engine:
    def __init__(self, obs_dims, local_q=None, *, num_units=64, batch_size=1024, max_episode_len=25,
                 capacity=int(1e6), num_envs=0, scenario="none", num_adversaries=0, lr=1e-2,
                 gamma=0.95, tau=1e-2, grad_clip=0.5, actor_reg=1e-3, adam_b1=0.9, adam_b2=0.999,
                 adam_eps=1e-8, seed=0, world_size=1, rank=0, device=None, episode_log_rows=0):
        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise RuntimeError("maddpg_amd runs on a ROCm GPU only (no CPU fallback)")
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        n = len(obs_dims)
        local_q = [False] * n if local_q is None else list(local_q)
        self.n = n
        self.obs_dims = [int(o) for o in obs_dims]
        self.local_q = [bool(x) for x in local_q]
        self.update_mode = "strict"
        self.num_units = int(num_units)
        self.batch_size = int(batch_size)
        self.max_episode_len = int(max_episode_len)
        self.capacity = int(capacity)
        self.num_envs = int(num_envs)
        self.scenario = scenario
        self.world_size, self.rank = int(world_size), int(rank)
        cfg = MdpConfig()
        cfg.n_agents = n
        for i in range(n):
            cfg.obs_dim[i] = self.obs_dims[i]
            cfg.local_q[i] = 1 if self.local_q[i] else 0
        cfg.act_dim = _lib.ACT_DIM
        cfg.num_units = self.num_units
        cfg.batch_size = self.batch_size
        cfg.max_episode_len = self.max_episode_len
        cfg.capacity = self.capacity
        cfg.num_envs = self.num_envs
        cfg.scenario = _lib.SCN[scenario]
        cfg.num_adversaries = int(num_adversaries)
        cfg.world_size, cfg.rank = self.world_size, self.rank
        cfg.lr, cfg.tau, cfg.grad_clip, cfg.actor_reg = lr, tau, grad_clip, actor_reg
        cfg.adam_b1, cfg.adam_b2, cfg.adam_eps = adam_b1, adam_b2, adam_eps
        cfg.gamma = float(gamma)
        cfg.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        cfg.episode_log_rows = int(episode_log_rows)
        self.cfg = cfg
        pt = ctypes.c_int64()
        nbytes = self.lib.mdp_arena_bytes(ctypes.byref(cfg), ctypes.byref(pt))
        if nbytes < 0:
            raise ValueError(f"invalid maddpg configuration: {self._config_error(cfg)}")
        self.param_floats = pt.value
        with torch.cuda.device(self.device):
            self.arena = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
            self.stream = torch.cuda.Stream(device=self.device)
            h = ctypes.c_void_p()
            rc = self.lib.mdp_create(ctypes.byref(cfg), ctypes.c_void_p(self.arena.data_ptr()), nbytes,
                                     ctypes.c_void_p(self.stream.cuda_stream), ctypes.byref(h))
        self.h = h
        if rc != 0:
            msg = self.lib.mdp_last_error(h).decode()
            self.lib.mdp_destroy(h)
            self.h = None
            raise ValueError(f"mdp_create failed: {msg}")
        lay = (ctypes.c_int32 * 6)()
        self.row_layout = []
        for i in range(n):
            self._c("mdp_row_layout", i, lay)
            self.row_layout.append(tuple(lay[:6]))
        self.row_stride = self.row_layout[0][5]
        self._tensors = {}
        for i in range(n):
            for net in (0, 1):
                infos = []
                for t in range(6):
                    ti = MdpTensorInfo()
                    self._c("mdp_tensor", i, net, t, ctypes.byref(ti))
                    infos.append((ti.offset, ti.rows, ti.cols, ti.dev_rows, ti.dev_cols))
                self._tensors[(i, net)] = infos

    # ------------------------------------------------------------ plumbing
    def _c(self, name, *args):
        rc = getattr(self.lib, name)(self.h, *args)
        return _lib.check(self.lib, self.h, rc, name)

    def _config_error(self, cfg):
        """why mdp_arena_bytes refused `cfg`: mdp_create validates the same layout
        first and keeps the message on the handle it returns (no GPU call)"""
        h = ctypes.c_void_p()
        self.lib.mdp_create(ctypes.byref(cfg), None, 0, None, ctypes.byref(h))
        msg = self.lib.mdp_last_error(h).decode() if h.value else "mdp_create returned no handle"
        self.lib.mdp_destroy(h)
        return msg

    def close(self):
        if getattr(self, "h", None):
            self.lib.mdp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync_in(self):
        """engine stream waits for work torch queued on the current stream"""
        self.stream.wait_stream(torch.cuda.current_stream(self.device))

    def sync_out(self):
        """torch's current stream waits for the engine stream"""
        torch.cuda.current_stream(self.device).wait_stream(self.stream)

    def synchronize(self):
        self._c("mdp_synchronize")

    @staticmethod
    def _ptr(t):
        """device pointer of a tensor for the C ABI (null for None).  A host tensor is
        refused: the kernels would dereference its address on the device."""
        if t is None:
            return ctypes.c_void_p(0)
        if not t.is_cuda:
            raise ValueError("the C ABI takes device tensors; got a host tensor")
        return ctypes.c_void_p(t.data_ptr())

    def region(self, name, dtype=torch.float32):
        off, nb = ctypes.c_int64(), ctypes.c_int64()
        self._c("mdp_region", _lib.REGION[name], ctypes.byref(off), ctypes.byref(nb))
        isz = torch.tensor([], dtype=dtype).element_size()
        return self.arena[off.value: off.value + (nb.value // isz) * isz].view(dtype)

    def net_tensors(self, agent, net):
        return self._tensors[(agent, net)]

    def grad_view(self, agent, net):
        """float32 view of one net's gradient in the GRAD region (all-reduce target)."""
        infos = self._tensors[(agent, net)]
        start = infos[0][0]
        end = infos[5][0] + ((infos[5][3] * infos[5][4] + 3) // 4) * 4
        return self.region("grad")[start:end]

    # ---------------------------------------------------------- parameters
    def _flat_shapes(self, agent, which):
        net = 1 if "critic" in which else 0
        return [(r, c) for (_o, r, c, _dr, _dc) in self._tensors[(agent, net)]]

    def set_params(self, agent, which, params):
        shapes = self._flat_shapes(agent, which)
        if isinstance(params, dict):
            parts = [np.asarray(params[k], np.float32).reshape(s) for k, s in zip(TENSOR_NAMES, shapes)]
            flat = np.concatenate([p.ravel() for p in parts])
        else:
            flat = np.asarray(params, np.float32).ravel()
        flat = np.ascontiguousarray(flat, np.float32)
        self._c("mdp_set_params", agent, _lib.WHICH[which], _lib.fptr(flat), flat.size)

    def get_params(self, agent, which):
        shapes = self._flat_shapes(agent, which)
        n = sum(r * c for r, c in shapes)
        flat = np.empty(n, np.float32)
        self._c("mdp_get_params", agent, _lib.WHICH[which], _lib.fptr(flat), n)
        out, s = {}, 0
        for k, (r, c) in zip(TENSOR_NAMES, shapes):
            a = flat[s:s + r * c].reshape(r, c)
            out[k] = a[0].copy() if k.startswith("b") else a.copy()
            s += r * c
        return out

    def get_beta_powers(self, agent, net):
        b = np.empty(2, np.float32)
        self._c("mdp_get_beta_powers", agent, net, _lib.fptr(b))
        return b

    def set_beta_powers(self, agent, net, b):
        b = np.ascontiguousarray(b, np.float32)
        self._c("mdp_set_beta_powers", agent, net, _lib.fptr(b))

    def init_params(self, seed=0):
        """tf.contrib.layers xavier_initializer (uniform) for all four nets per
        agent, each drawn independently (targets are NOT copies: maddpg.py:66,104)."""
        rng = np.random.default_rng(seed)
        H = self.num_units
        for i in range(self.n):
            for which in ("actor", "critic", "tgt_actor", "tgt_critic"):
                shapes = self._flat_shapes(i, which)
                p = {}
                for k, (r, c) in zip(TENSOR_NAMES, shapes):
                    if k.startswith("W"):
                        lim = np.sqrt(6.0 / (r + c))
                        p[k] = rng.uniform(-lim, lim, size=(r, c)).astype(np.float32)
                    else:
                        p[k] = np.zeros((r, c), np.float32)
                self.set_params(i, which, p)
        return H

    # --------------------------------------------------------- checkpoint
    SETS = ("actor", "critic", "tgt_actor", "tgt_critic", "m_actor", "v_actor", "m_critic", "v_critic")

    def state_dict(self):
        """Every variable tf.train.Saver would save (tf_util.py:259-273): weights,
        targets, Adam slots and beta powers, keyed like the TF1 scopes."""
        out = {}
        for i in range(self.n):
            for w in self.SETS:
                for k, v in self.get_params(i, w).items():
                    out[f"agent_{i}/{w}/{k}"] = v
            out[f"agent_{i}/actor/beta_power"] = self.get_beta_powers(i, 0)
            out[f"agent_{i}/critic/beta_power"] = self.get_beta_powers(i, 1)
        return out

    def load_state_dict(self, sd):
        for i in range(self.n):
            for w in self.SETS:
                self.set_params(i, w, {k: sd[f"agent_{i}/{w}/{k}"] for k in TENSOR_NAMES})
            self.set_beta_powers(i, 0, sd[f"agent_{i}/actor/beta_power"])
            self.set_beta_powers(i, 1, sd[f"agent_{i}/critic/beta_power"])

    @staticmethod
    def checkpoint_path(fname):
        if fname.endswith(".npz"):
            return fname
        if fname.endswith("/") or os.path.isdir(fname):
            return os.path.join(fname, "maddpg_amd_state.npz")
        return fname + ".npz"

    def save_state(self, fname, fmt="npz"):
        """fmt "npz": one .npz keyed like state_dict(); fmt "tf1": a TF1 tensor
        bundle at prefix `fname` with the reference's variable names, as
        tf.train.Saver().save(sess, fname) writes it (tf_util.py:267-273;
        `fname`.index + `fname`.data-00000-of-00001 + the `checkpoint` state
        file; no .meta -- the graph is built by code on both sides)."""
        if fmt == "tf1":
            from .common import tf_checkpoint as tfc
            self._drop_stale(fname, keep="tf1")
            tfc.write_bundle(fname, tfc.tf1_from_state(self.state_dict()))
            d = os.path.dirname(os.path.abspath(fname + "x"))
            with open(os.path.join(d, "checkpoint"), "w") as fh:
                p = os.path.abspath(fname) + ("/" if fname.endswith("/") else "")
                fh.write(f'model_checkpoint_path: "{p}"\nall_model_checkpoint_paths: "{p}"\n')
            return fname
        if fmt != "npz":
            raise ValueError(f"unknown checkpoint format {fmt!r} (npz, tf1)")
        path = self.checkpoint_path(fname)
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        self._drop_stale(fname, keep="npz")
        np.savez(path, **self.state_dict())
        return path

    def _drop_stale(self, fname, keep):
        """a save in one format removes the other format's files at the same
        prefix, so a later --restore cannot pick up an older checkpoint"""
        if keep == "npz":
            for f in (fname + ".index", fname + ".data-00000-of-00001"):
                if os.path.isfile(f):
                    os.remove(f)
        elif os.path.isfile(self.checkpoint_path(fname)):
            os.remove(self.checkpoint_path(fname))

    def load_state(self, fname):
        """Restore from a TF1 tensor bundle at prefix `fname` (the reference's
        tf.train.Saver checkpoint, tf_util.py:259-264) or from the .npz
        save_state writes.  save_state removes the other format's files, so
        both exist only when another tool wrote one of them: then the newer
        one (nanosecond modification times) is read; on a tie (a copy that
        kept timestamps, a tar archive's whole-second times) the TF1 bundle,
        the reference's own format, is read and a warning names the choice."""
        from .common import tf_checkpoint as tfc
        path = self.checkpoint_path(fname)
        if tfc.is_bundle(fname) and os.path.isfile(path):
            t_npz, t_tf1 = os.stat(path).st_mtime_ns, os.stat(fname + ".index").st_mtime_ns
            if t_npz == t_tf1:
                import warnings
                warnings.warn(f"both {path} and the TF1 bundle {fname}.index exist with the same modification "
                              f"time; restoring the TF1 bundle (remove it to restore the .npz)")
            use_tf1 = t_tf1 >= t_npz
        else:
            use_tf1 = tfc.is_bundle(fname)
        if use_tf1:
            self.load_state_dict(tfc.state_from_tf1(tfc.read_bundle(fname), self.n, self.SETS))
            return fname
        with np.load(path, allow_pickle=False) as z:
            self.load_state_dict({k: z[k] for k in z.files})
        return path

    # ------------------------------------------------------------- replay
    def buffer_len(self):
        return int(self.lib.mdp_buffer_len(self.h))

    def add_rows(self, rows):
        rows = rows.to(self.device, torch.float32).contiguous()
        assert rows.dim() == 2 and rows.shape[1] == self.row_stride
        self.sync_in()
        self._c("mdp_buffer_add_rows", self._ptr(rows), rows.shape[0])
        self._keep = rows  # keep alive until the stream consumed it
        self.sync_out()

    def put_agent(self, agent, pos, cols):
        pos = pos.to(self.device, torch.int64).contiguous()
        cols = cols.to(self.device, torch.float32).contiguous()
        self.sync_in()
        self._c("mdp_buffer_put_agent", agent, self._ptr(pos), self._ptr(cols), pos.shape[0])
        self.sync_out()

    def set_ring(self, length, next_idx):
        self._c("mdp_buffer_set_len", int(length), int(next_idx))

    def seed_py_random(self, seed):
        self._c("mdp_seed_py_random", int(seed) & 0xFFFFFFFFFFFFFFFF)

    def set_rng_state(self, state625):
        st = np.ascontiguousarray(np.asarray(state625, dtype=np.uint64).astype(np.uint32))
        assert st.size == 625
        self._c("mdp_set_rng_state", st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))

    def get_rng_state(self):
        st = np.empty(625, np.uint32)
        self._c("mdp_get_rng_state", st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
        return st

    def make_index(self, count, out=None):
        if out is None:
            out = torch.empty(count, dtype=torch.int32, device=self.device)
        self.sync_in()
        self._c("mdp_make_index", int(count), self._ptr(out))
        self.sync_out()
        return out

    def sample_rows(self, idx, out=None):
        idx = idx.to(self.device, torch.int32).contiguous()
        if out is None:
            out = torch.empty((idx.shape[0], self.row_stride), dtype=torch.float32, device=self.device)
        self.sync_in()
        self._c("mdp_sample_rows", self._ptr(idx), idx.shape[0], self._ptr(out))
        self.sync_out()
        return out

    # ------------------------------------------------------------ policies
    def act(self, agent, obs, target=False, u=None):
        obs = obs.to(self.device, torch.float32).contiguous()
        out = torch.empty((obs.shape[0], _lib.ACT_DIM), dtype=torch.float32, device=self.device)
        if u is not None:
            u = u.to(self.device, torch.float32).contiguous()
        self.sync_in()
        self._c("mdp_act", agent, 1 if target else 0, self._ptr(obs), self._ptr(out), obs.shape[0], self._ptr(u))
        self.sync_out()
        return out

    def actor_logits(self, agent, obs, target=False):
        obs = obs.to(self.device, torch.float32).contiguous()
        out = torch.empty((obs.shape[0], _lib.ACT_DIM), dtype=torch.float32, device=self.device)
        self.sync_in()
        self._c("mdp_actor_logits", agent, 1 if target else 0, self._ptr(obs), self._ptr(out), obs.shape[0])
        self.sync_out()
        return out

    def q_values(self, agent, x, target=False):
        x = x.to(self.device, torch.float32).contiguous()
        out = torch.empty(x.shape[0], dtype=torch.float32, device=self.device)
        self.sync_in()
        self._c("mdp_q_values", agent, 1 if target else 0, self._ptr(x), self._ptr(out), x.shape[0])
        self.sync_out()
        return out

    # ------------------------------------------------------------ training
    @staticmethod
    def _sized(what, t, want):
        """the C side reads exactly `want` elements of an injected index / noise
        tensor: a short one would be an out-of-bounds device read, so refuse it"""
        if t is not None and t.numel() != want:
            raise ValueError(f"{what}: {t.numel()} elements, the update reads {want}")

    def update(self, agent, idx=None, u_tgt=None, u_act=None):
        B, n, A = self.batch_size, self.n, _lib.ACT_DIM
        self._sized("idx", idx, B)
        self._sized("u_tgt", u_tgt, n * B * A)
        self._sized("u_act", u_act, B * A)
        args = []
        for t, dt in ((idx, torch.int32), (u_tgt, torch.float32), (u_act, torch.float32)):
            args.append(None if t is None else t.to(self.device, dt).contiguous())
        self.sync_in()
        self._c("mdp_update", agent, *[self._ptr(a) for a in args])
        self._keep = args
        self.sync_out()

    UPDATE_MODES = {"strict": 0, "throughput": 1}

    def set_update_mode(self, mode):
        """'strict' (the reference's order, default) or 'throughput' (every
        agent's gradients from the round-start parameters, then every optimizer
        step: SURVEY.md 8e, not the reference's semantics).  mdp_set_update_mode."""
        self._c("mdp_set_update_mode", self.UPDATE_MODES[mode])
        self.update_mode = mode

    def update_all(self, idx=None, u_tgt=None, u_act=None):
        """one throughput-mode round; idx [n, B], u_tgt [n, n, B, 5], u_act [n, B, 5]
        (injected randomness for parity; None: device streams).  mdp_update_all."""
        B, n, A = self.batch_size, self.n, _lib.ACT_DIM
        self._sized("idx", idx, n * B)
        self._sized("u_tgt", u_tgt, n * n * B * A)
        self._sized("u_act", u_act, n * B * A)
        args = []
        for t, dt in ((idx, torch.int32), (u_tgt, torch.float32), (u_act, torch.float32)):
            args.append(None if t is None else t.to(self.device, dt).contiguous())
        self.sync_in()
        self._c("mdp_update_all", *[self._ptr(a) for a in args])
        self._keep = args
        self.sync_out()

    def agent_update(self, agent, t, idx=None, u=None):
        """MADDPGAgentTrainer.update(agents, t) in one C call (mdp_agent_update):
        None below the gates (maddpg.py:162-165), else the 6 stats.  u: None or
        [n * B * 5 target-actor uniforms | B * 5 actor-loss uniforms] (flat)."""
        B, n, A = self.batch_size, self.n, _lib.ACT_DIM
        self._sized("idx", idx, B)
        self._sized("u", u, (n + 1) * B * A)
        args = []
        for a, dt in ((idx, torch.int32), (u, torch.float32)):
            args.append(None if a is None else a.to(self.device, dt).contiguous().reshape(-1))
        out = (ctypes.c_double * 6)()
        self.sync_in()
        rc = self._c("mdp_agent_update", int(agent), int(t), *[self._ptr(a) for a in args], out)
        self._keep = args
        self.sync_out()
        return None if rc == 1 else update_stats(out)

    def update_gate(self, t):
        return self._c("mdp_update_gate", int(t))

    def update_round(self):
        self._c("mdp_update_round")

    def train_step(self, rounds):
        """one vector env step + `rounds` update rounds, as one graph replay
        (mdp_train_step; single-GPU path)."""
        self._c("mdp_train_step", int(rounds))

    def train_steps(self, rounds, launch=True):
        """len(rounds) consecutive vector steps (step i: rollout + rounds[i] update
        rounds) as ONE graph replay (mdp_train_steps); launch=False only
        captures and instantiates that graph ahead of time."""
        ks = (ctypes.c_int32 * len(rounds))(*[int(k) for k in rounds])
        self._c("mdp_train_steps", len(rounds), ks, 1 if launch else 0)

    def dp_init(self, world, rank, uid=None):
        """Native data parallelism: join an RCCL communicator of `world` ranks
        (mdp_dp_init).  `uid` (128 bytes) comes from rank 0's dp_unique_id();
        with torch.distributed initialised, dp_init_from_dist() shares it."""
        if uid is None:
            uid = Engine.dp_unique_id()
        self._c("mdp_dp_init", bytes(uid), int(world), int(rank))

    @staticmethod
    def dp_unique_id():
        buf = ctypes.create_string_buffer(128)
        if _lib.load().mdp_dp_unique_id(buf) != 0:
            raise _lib.MdpError("mdp_dp_unique_id failed (librccl.so.1 not loadable?)")
        return buf.raw

    def dp_init_from_dist(self, world, rank):
        """rank 0 makes the RCCL id, torch.distributed broadcasts it, every rank
        joins; returns False on every rank if rank 0 could not make one."""
        import torch.distributed as dist
        obj = [None]
        if rank == 0:
            try:
                obj[0] = Engine.dp_unique_id()
            except Exception:
                obj[0] = None
        dist.broadcast_object_list(obj, src=0)
        if obj[0] is None:
            return False
        self.dp_init(world, rank, obj[0])
        return True

    def dp_xgmi_open(self, world, rank):
        """export this rank's exchange buffer; returns its 64-byte IPC handle"""
        buf = ctypes.create_string_buffer(64)
        self._c("mdp_dp_xgmi_open", int(world), int(rank), buf)
        return buf.raw

    def dp_xgmi_connect(self, handles):
        self._c("mdp_dp_xgmi_connect", b"".join(bytes(x) for x in handles))

    def dp_xgmi_probe(self):
        bad = ctypes.c_int32(0)
        self._c("mdp_dp_xgmi_probe", ctypes.byref(bad))
        return bad.value

    def dp_xgmi_init_from_dist(self, world, rank):
        """Direct xGMI gradient exchange (mdp_dp_xgmi_*): the handshake of
        parallel.xgmi_handshake over torch.distributed.  Returns False
        (everything torn down on every rank) when any rank failed, so the
        caller can fall back to dp_init_from_dist."""
        from .parallel import xgmi_handshake
        eng = self

        class _Ops:
            device = eng.device
            open = staticmethod(eng.dp_xgmi_open)
            connect = staticmethod(eng.dp_xgmi_connect)
            probe = staticmethod(eng.dp_xgmi_probe)

            @staticmethod
            def enable():
                eng._c("mdp_dp_xgmi_enable")

            @staticmethod
            def close():
                eng._c("mdp_dp_xgmi_close")

        ok, err = xgmi_handshake(_Ops, world, rank)
        if not ok and err is not None:
            import sys
            print(f"[rank {rank}] xGMI exchange unavailable ({err}); using RCCL", file=sys.stderr)
        return ok

    DP_KINDS = {0: None, 1: "rccl", 2: "xgmi"}

    def dp_info(self):
        """{kind, ranks, rank, peers}: the communicator this rank's gradient
        exchange runs over (mdp_dp_info)."""
        out = (ctypes.c_int32 * 4)()
        self._c("mdp_dp_info", out)
        return {"kind": self.DP_KINDS[out[0]], "ranks": out[1], "rank": out[2], "peers": out[3]}

    def dp_exchange_stats(self, reset=False):
        """direct xGMI exchange wait of this rank's chunk workgroups since the
        last reset (mdp_dp_exchange_stats): {chunk_exchanges, mean_us, max_us,
        total_us}."""
        out = (ctypes.c_double * 4)()
        self._c("mdp_dp_exchange_stats", out, 1 if reset else 0)
        return {"chunk_exchanges": int(out[0]), "mean_us": out[1], "max_us": out[2], "total_us": out[3]}

    def dp_exchange_stats_enable(self, on=True):
        """stamp the xGMI exchange waits in the optimizer launches issued while
        enabled (mdp_dp_exchange_stats_enable; default off)"""
        self._c("mdp_dp_exchange_stats_enable", 1 if on else 0)

    def param_checksum(self):
        """exact fingerprint of every replicated state region (weights, targets,
        Adam moments, beta powers): int64 sums of the raw 32-bit words, plus a
        position-weighted sum so permutations differ"""
        out = []
        for name in ("theta", "target", "adam_m", "adam_v", "beta"):
            w = self.region(name, torch.int32).to(torch.int64)
            pos = torch.arange(1, w.numel() + 1, device=w.device, dtype=torch.int64)
            out += [int(w.sum().item()), int(((w & 0xFFFF) * pos).sum().item())]
        return out

    def set_graphs(self, on=True):
        """hipGraph replay of update_round (default on; per-kernel profiling runs eager)."""
        self._c("mdp_set_graphs", 1 if on else 0)

    def critic_grad(self, agent, idx, u_tgt=None):
        B, n, A = self.batch_size, self.n, _lib.ACT_DIM
        self._sized("idx", idx, B)
        self._sized("u_tgt", u_tgt, n * B * A)
        idx = idx.to(self.device, torch.int32).contiguous()
        u_tgt = None if u_tgt is None else u_tgt.to(self.device, torch.float32).contiguous()
        self._c("mdp_critic_grad", agent, self._ptr(idx), self._ptr(u_tgt))
        self._keep = (idx, u_tgt)

    def actor_grad(self, agent, idx, u_act=None):
        B, A = self.batch_size, _lib.ACT_DIM
        self._sized("idx", idx, B)
        self._sized("u_act", u_act, B * A)
        idx = idx.to(self.device, torch.int32).contiguous()
        u_act = None if u_act is None else u_act.to(self.device, torch.float32).contiguous()
        self._c("mdp_actor_grad", agent, self._ptr(idx), self._ptr(u_act))
        self._keep = (idx, u_act)

    def reduce_grad(self, agent, net):
        self._c("mdp_reduce_grad", agent, net)

    def apply_grad(self, agent, net, scale=1.0):
        self._c("mdp_apply_grad", agent, net, float(scale))

    def index_slot(self, agent):
        """int32 view of the device index slot used by agent's update this round."""
        return self.region("index", torch.int32)[agent * self.batch_size:(agent + 1) * self.batch_size]

    def stats(self, agent):
        out = (ctypes.c_double * 6)()
        self._c("mdp_get_stats", agent, out)
        return list(out)

    def check_finite(self):
        """NaN / Inf values in every parameter set (weights, targets, Adam m, v)
        and in the agents' update stats, counted on the device (mdp_check_finite:
        the reference's opt-in check_nan, tf_util.py:322,366-368)"""
        out = ctypes.c_int64()
        self._c("mdp_check_finite", ctypes.byref(out))
        return int(out.value)

    def stats_future(self, agent):
        """Snapshot of agent's 6 update stats, copied D2H in stream order (no sync);
        returns (host tensor, event) -- wait on the event before reading."""
        src = self.region("stats", torch.float64)[agent * 8:agent * 8 + 6]
        dst = torch.empty(6, dtype=torch.float64, pin_memory=True)
        with torch.cuda.stream(self.stream):
            dst.copy_(src, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return dst, ev

    # ----------------------------------------------------------------- env
    @property
    def n_entities(self):
        """agents + landmarks (scenario make_world)."""
        landmarks = {"simple": 1, "simple_spread": self.n, "simple_adversary": self.n - 1,
                     "simple_tag": 2}.get(self.scenario, 0)
        return self.n + landmarks

    def env_reset(self):
        self._c("mdp_env_reset")

    def env_step(self, act_in=None, u=None):
        a = None if act_in is None else act_in.to(self.device, torch.float32).contiguous()
        uu = None if u is None else u.to(self.device, torch.float32).contiguous()
        if a is not None or uu is not None:
            self.sync_in()
        self._c("mdp_env_step", self._ptr(a), self._ptr(uu))
        if a is not None or uu is not None:
            self._keep = (a, uu)
            self.sync_out()

    def env_step_bench(self, out=None):
        """one vector env step (policy actions) that also returns every agent's
        scenario benchmark_data() record, [E, n, BENCH_W] float32 on the device
        (mdp_env_step_bench; --benchmark mode, train.py:139-141)."""
        if out is None:
            out = torch.empty((self.num_envs, self.n, _lib.BENCH_W), dtype=torch.float32, device=self.device)
        self._c("mdp_env_step_bench", self._ptr(out))
        self.sync_out()
        return out

    def env_state(self):
        E, ne = self.num_envs, self.n_entities
        pos = np.empty((E, ne, 2), np.float32)
        vel = np.empty((E, ne, 2), np.float32)
        goal = np.empty(E, np.int32)
        step = np.empty(E, np.int32)
        self._c("mdp_env_get_state", _lib.fptr(pos), _lib.fptr(vel),
                goal.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                step.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        return {"pos": pos, "vel": vel, "goal": goal, "ep_step": step}

    def set_env_state(self, pos, vel, goal=None, ep_step=None):
        E = self.num_envs
        pos = np.ascontiguousarray(pos, np.float32)
        vel = np.ascontiguousarray(vel, np.float32)
        goal = np.ascontiguousarray(np.zeros(E) if goal is None else goal, np.int32)
        ep_step = np.ascontiguousarray(np.zeros(E) if ep_step is None else ep_step, np.int32)
        self._c("mdp_env_set_state", _lib.fptr(pos), _lib.fptr(vel),
                goal.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                ep_step.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))

    def env_obs(self):
        out = torch.empty((self.num_envs, sum(self.obs_dims)), dtype=torch.float32, device=self.device)
        self._c("mdp_env_obs", self._ptr(out))
        self.sync_out()
        return out

    def episode_count(self):
        n = self.lib.mdp_episode_count(self.h)
        if n < 0:
            raise _lib.MdpError("mdp_episode_count failed")
        return int(n)

    def episode_log(self, first, n):
        out = np.empty((n, 1 + self.n), np.float32)
        if n:
            self._c("mdp_episode_log", int(first), int(n), _lib.fptr(out))
        return out

    def replay_rows(self, start, count):
        """float32 view [count, row_stride] of the replay region (no copy)."""
        r = self.region("replay")
        return r[start * self.row_stride:(start + count) * self.row_stride].view(count, self.row_stride)

    # ---------------------------------------------------------- profiling
    def prof_enable(self, kind, on=True):
        self._c("mdp_prof_enable", _lib.KERNEL[kind], 1 if on else 0)

    def prof_read(self, kind):
        ms, n = ctypes.c_double(), ctypes.c_int64()
        self._c("mdp_prof_read", _lib.KERNEL[kind], ctypes.byref(ms), ctypes.byref(n))
        return ms.value, n.value
