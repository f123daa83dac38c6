"""ctypes binding of libmaddpg_hip.so (C ABI in include/maddpg_hip.h).

This is the binding a maintainer adds on the reference side (there is no FFI
in the pure-Python reference).  torch is imported first so
the library resolves ``libamdhip64.so.7`` to the HIP runtime torch already
loaded (one runtime per process: device pointers and streams are shared).

There is deliberately NO fallback: if the shared library is missing or fails
to load, importing the product path raises.
"""
import ctypes
import os
import re

import torch  # noqa: F401  (load torch's HIP runtime before ours)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MDP_LIB") or os.path.join(HERE, "libmaddpg_hip.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "maddpg_hip.h")

MAX_AGENTS = 8
ACT_DIM = 5
BENCH_W = 8   # MDP_BENCH_W: floats per agent benchmark_data record
MAX_UNITS = 256  # MDP_MAX_UNITS: largest --num-units
ABI_VERSION = 5

SCN = {"none": 0, "simple": 1, "simple_spread": 2, "simple_adversary": 3, "simple_tag": 4}
WHICH = {"actor": 0, "critic": 1, "tgt_actor": 2, "tgt_critic": 3, "m_actor": 4, "v_actor": 5,
         "m_critic": 6, "v_critic": 7, "g_actor": 8, "g_critic": 9}
REGION = {"theta": 0, "target": 1, "adam_m": 2, "adam_v": 3, "grad": 4, "replay": 5, "index": 6,
          "stats": 7, "env": 8, "eplog": 9, "beta": 10, "slab": 11, "ctl": 12}
KERNEL = {"index": 0, "gather": 1, "critic_grad": 2, "actor_grad": 3, "apply": 4, "rollout": 5,
          "reduce": 6, "reduce_apply": 7, "allreduce": 8}


class MdpConfig(ctypes.Structure):
    _fields_ = [
        ("n_agents", ctypes.c_int32),
        ("obs_dim", ctypes.c_int32 * MAX_AGENTS),
        ("local_q", ctypes.c_int32 * MAX_AGENTS),
        ("act_dim", ctypes.c_int32),
        ("num_units", ctypes.c_int32),
        ("batch_size", ctypes.c_int32),
        ("max_episode_len", ctypes.c_int32),
        ("capacity", ctypes.c_int64),
        ("num_envs", ctypes.c_int32),
        ("scenario", ctypes.c_int32),
        ("num_adversaries", ctypes.c_int32),
        ("world_size", ctypes.c_int32),
        ("rank", ctypes.c_int32),
        ("lr", ctypes.c_float),
        ("tau", ctypes.c_float),
        ("grad_clip", ctypes.c_float),
        ("actor_reg", ctypes.c_float),
        ("adam_b1", ctypes.c_float),
        ("adam_b2", ctypes.c_float),
        ("adam_eps", ctypes.c_float),
        ("gamma", ctypes.c_double),
        ("seed", ctypes.c_uint64),
        ("episode_log_rows", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


class MdpTensorInfo(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_int64), ("rows", ctypes.c_int32), ("cols", ctypes.c_int32),
                ("dev_rows", ctypes.c_int32), ("dev_cols", ctypes.c_int32)]


_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_F32P = ctypes.POINTER(ctypes.c_float)
_F64P = ctypes.POINTER(ctypes.c_double)
_U32P = ctypes.POINTER(ctypes.c_uint32)
_I32P = ctypes.POINTER(ctypes.c_int32)

# name -> (restype, argtypes); device pointers are passed as c_void_p
SIGNATURES = {
    "mdp_abi_version": (_I32, []),
    "mdp_arena_bytes": (_I64, [ctypes.POINTER(MdpConfig), ctypes.POINTER(_I64)]),
    "mdp_create": (ctypes.c_int, [ctypes.POINTER(MdpConfig), _P, _I64, _P, ctypes.POINTER(_P)]),
    "mdp_destroy": (ctypes.c_int, [_P]),
    "mdp_last_error": (ctypes.c_char_p, [_P]),
    "mdp_stream": (_P, [_P]),
    "mdp_synchronize": (ctypes.c_int, [_P]),
    "mdp_region": (ctypes.c_int, [_P, _I32, ctypes.POINTER(_I64), ctypes.POINTER(_I64)]),
    "mdp_tensor": (ctypes.c_int, [_P, _I32, _I32, _I32, ctypes.POINTER(MdpTensorInfo)]),
    "mdp_row_layout": (ctypes.c_int, [_P, _I32, _I32P]),
    "mdp_set_params": (ctypes.c_int, [_P, _I32, _I32, _F32P, _I64]),
    "mdp_get_params": (ctypes.c_int, [_P, _I32, _I32, _F32P, _I64]),
    "mdp_get_beta_powers": (ctypes.c_int, [_P, _I32, _I32, _F32P]),
    "mdp_set_beta_powers": (ctypes.c_int, [_P, _I32, _I32, _F32P]),
    "mdp_buffer_len": (_I64, [_P]),
    "mdp_buffer_add_rows": (ctypes.c_int, [_P, _P, _I64]),
    "mdp_buffer_put_agent": (ctypes.c_int, [_P, _I32, _P, _P, _I64]),
    "mdp_buffer_set_len": (ctypes.c_int, [_P, _I64, _I64]),
    "mdp_seed_py_random": (ctypes.c_int, [_P, ctypes.c_uint64]),
    "mdp_set_rng_state": (ctypes.c_int, [_P, _U32P]),
    "mdp_get_rng_state": (ctypes.c_int, [_P, _U32P]),
    "mdp_make_index": (ctypes.c_int, [_P, _I32, _P]),
    "mdp_sample_rows": (ctypes.c_int, [_P, _P, _I32, _P]),
    "mdp_act": (ctypes.c_int, [_P, _I32, _I32, _P, _P, _I32, _P]),
    "mdp_actor_logits": (ctypes.c_int, [_P, _I32, _I32, _P, _P, _I32]),
    "mdp_q_values": (ctypes.c_int, [_P, _I32, _I32, _P, _P, _I32]),
    "mdp_update": (ctypes.c_int, [_P, _I32, _P, _P, _P]),
    "mdp_update_gate": (ctypes.c_int, [_P, _I64]),
    "mdp_update_round": (ctypes.c_int, [_P]),
    "mdp_set_graphs": (ctypes.c_int, [_P, _I32]),
    "mdp_train_step": (ctypes.c_int, [_P, _I32]),
    "mdp_dp_unique_id": (ctypes.c_int, [ctypes.c_char_p]),
    "mdp_grad_variant": (ctypes.c_int, [_P, _I32]),
    "mdp_dp_init": (ctypes.c_int, [_P, ctypes.c_char_p, _I32, _I32]),
    "mdp_dp_xgmi_open": (ctypes.c_int, [_P, _I32, _I32, ctypes.c_char_p]),
    "mdp_dp_xgmi_connect": (ctypes.c_int, [_P, ctypes.c_char_p]),
    "mdp_dp_xgmi_probe": (ctypes.c_int, [_P, _I32P]),
    "mdp_dp_xgmi_enable": (ctypes.c_int, [_P]),
    "mdp_dp_xgmi_close": (ctypes.c_int, [_P]),
    "mdp_dp_info": (ctypes.c_int, [_P, _I32P]),
    "mdp_dp_exchange_stats": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double), _I32]),
    "mdp_dp_exchange_stats_enable": (ctypes.c_int, [_P, _I32]),
    "mdp_train_steps": (ctypes.c_int, [_P, _I32, ctypes.POINTER(ctypes.c_int32), _I32]),
    "mdp_agent_update": (ctypes.c_int, [_P, _I32, ctypes.c_int64, _P, _P, ctypes.POINTER(ctypes.c_double)]),
    "mdp_ra_plan": (ctypes.c_int, [ctypes.POINTER(MdpConfig), _I32, _I32, _I32P]),
    "mdp_critic_grad": (ctypes.c_int, [_P, _I32, _P, _P]),
    "mdp_actor_grad": (ctypes.c_int, [_P, _I32, _P, _P]),
    "mdp_reduce_grad": (ctypes.c_int, [_P, _I32, _I32]),
    "mdp_apply_grad": (ctypes.c_int, [_P, _I32, _I32, ctypes.c_float]),
    "mdp_get_stats": (ctypes.c_int, [_P, _I32, _F64P]),
    "mdp_check_finite": (ctypes.c_int, [_P, ctypes.POINTER(_I64)]),
    "mdp_env_reset": (ctypes.c_int, [_P]),
    "mdp_env_step": (ctypes.c_int, [_P, _P, _P]),
    "mdp_env_get_state": (ctypes.c_int, [_P, _F32P, _F32P, _I32P, _I32P]),
    "mdp_env_set_state": (ctypes.c_int, [_P, _F32P, _F32P, _I32P, _I32P]),
    "mdp_env_obs": (ctypes.c_int, [_P, _P]),
    "mdp_env_step_bench": (ctypes.c_int, [_P, _P]),
    "mdp_set_update_mode": (ctypes.c_int, [_P, _I32]),
    "mdp_update_all": (ctypes.c_int, [_P, _P, _P, _P]),
    "mdp_episode_count": (_I64, [_P]),
    "mdp_episode_log": (ctypes.c_int, [_P, _I64, _I64, _F32P]),
    "mdp_prof_enable": (ctypes.c_int, [_P, _I32, _I32]),
    "mdp_prof_read": (ctypes.c_int, [_P, _I32, _F64P, ctypes.POINTER(_I64)]),
}


def header_symbols(path=HEADER):
    """Function names declared in include/maddpg_hip.h."""
    text = open(path).read()
    return sorted(set(re.findall(r"\b(mdp_[a-z0-9_]+)\s*\(", text)))


_lib = None


def load():
    """Load and type the library (raises if it is missing: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make -C maddpg_amd/csrc` "
            "(or __graft_entry__.build()); maddpg_amd has no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        if os.environ.get("MDP_LIB") and not hasattr(lib, name):
            continue  # an explicitly chosen other build (A/B of an older one): entry points it lacks stay unbound
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.mdp_abi_version() != ABI_VERSION:
        raise ImportError("libmaddpg_hip.so ABI version mismatch")
    _lib = lib
    return lib


class MdpError(RuntimeError):
    pass


def check(lib, handle, rc, what=""):
    if rc < 0:
        msg = lib.mdp_last_error(handle)
        raise MdpError(f"{what}: {msg.decode() if msg else 'error'}")
    return rc


def fptr(a):
    """float* of a contiguous float32 numpy array."""
    return a.ctypes.data_as(_F32P)
