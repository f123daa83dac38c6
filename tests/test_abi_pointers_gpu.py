"""The C ABI refuses host pointers itself (round 5's r05h fault).

A ctypes binding written against include/maddpg_hip.h -- INTEGRATION.md's --
that hands the library a CPU tensor's address gets -1 and a message from the
entry point, not an illegal memory access in a kernel; the handle stays usable.
Device memory from PyTorch's caching allocator is accepted in both of its
modes: plain hipMalloc segments and expandable (virtual-memory) segments.
(tests/native/abi_host_check.cpp covers every entry point from C++.)
"""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no ROCm GPU", allow_module_level=True)

from maddpg_amd.engine import Engine  # noqa: E402
from tests.helpers import joint_rows, synthetic_trainer_case  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _engine(B=256, L=1200, seed=3):
    dims = [18, 18, 18]
    c = synthetic_trainer_case(dims, B, L, seed=seed)
    eng = Engine(dims, batch_size=B, capacity=L)
    eng.add_rows(torch.from_numpy(joint_rows(c["data"], dims)))
    eng.init_params(0)
    return eng, c


def test_raw_binding_host_pointers_refused_not_faulted():
    eng, c = _engine()
    lib, h = eng.lib, eng.h
    idx_host = torch.from_numpy(c["idx"][0].astype(np.int32))           # a CPU tensor
    u_host = torch.zeros(eng.n * eng.batch_size * 5, dtype=torch.float32)
    out_host = torch.zeros(eng.batch_size * eng.row_stride, dtype=torch.float32)
    p = lambda t: ctypes.c_void_p(t.data_ptr())                          # noqa: E731 (no Engine._ptr guard)
    calls = [("mdp_update", (0, p(idx_host), None, None)),
             ("mdp_critic_grad", (0, p(idx_host), None)),
             ("mdp_actor_grad", (1, p(idx_host), None)),
             ("mdp_sample_rows", (p(idx_host), eng.batch_size, p(out_host))),
             ("mdp_make_index", (eng.batch_size, p(idx_host))),
             ("mdp_update", (0, None, p(u_host), None))]
    for name, args in calls:
        rc = getattr(lib, name)(h, *args)
        msg = lib.mdp_last_error(h).decode()
        assert rc < 0, name
        assert "not device memory" in msg and name in msg, (name, msg)
    # nothing was launched, nothing faulted; the same handle trains on device indices
    eng.synchronize()
    eng.update(0, idx=torch.from_numpy(c["idx"][0]), u_tgt=torch.from_numpy(c["u_tgt"][0]),
               u_act=torch.from_numpy(c["u_act"][0]))
    eng.synchronize()
    assert all(np.isfinite(eng.stats(0)))


def test_device_buffer_shorter_than_the_call_refused():
    """B - 1 indices at the very end of a hipMalloc allocation: mdp_update would
    read one int past it.  Run only where the runtime reports the allocation's
    exact extent (the library checks with the same hipMemGetAddressRange), so a
    runtime that rounds extents can never let the kernel read past a mapping."""
    eng, c = _engine()
    hip = eng.lib        # the HIP runtime the library itself links (resolved through its dependencies)
    nbytes = 4 << 20
    base = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(base), ctypes.c_size_t(nbytes)) == 0
    try:
        rb, ext = ctypes.c_void_p(), ctypes.c_size_t()
        exact = (hip.hipMemGetAddressRange(ctypes.byref(rb), ctypes.byref(ext), base) == 0
                 and rb.value == base.value and ext.value == nbytes)
        if not exact:
            pytest.skip(f"runtime reports extent {ext.value} for a {nbytes}-byte allocation")
        tail = ctypes.c_void_p(base.value + nbytes - 4 * (eng.batch_size - 1))
        rc = eng.lib.mdp_update(eng.h, 0, tail, None, None)
        msg = eng.lib.mdp_last_error(eng.h).decode()
        assert rc < 0 and "allocation too small" in msg, msg
        # exactly B indices ending at the allocation's end are accepted
        zeros = torch.zeros(eng.batch_size, dtype=torch.int32, device="cuda")
        full = ctypes.c_void_p(base.value + nbytes - 4 * eng.batch_size)
        assert hip.hipMemcpy(full, ctypes.c_void_p(zeros.data_ptr()), ctypes.c_size_t(4 * eng.batch_size), 3) == 0
        eng.lib.mdp_update.restype = ctypes.c_int
        assert eng.lib.mdp_update(eng.h, 0, full, None, None) == 0, eng.lib.mdp_last_error(eng.h).decode()
        eng.synchronize()
    finally:
        torch.cuda.synchronize()
        hip.hipFree(base)


CHILD = r"""
import json, os, sys, numpy as np, torch
sys.path.insert(0, os.environ["ROOT"])
from maddpg_amd.engine import Engine
from tests.helpers import joint_rows, synthetic_trainer_case
dims, B, L = [18, 18, 18], 256, 1200
c = synthetic_trainer_case(dims, B, L, seed=4)
eng = Engine(dims, batch_size=B, capacity=L)
eng.add_rows(torch.from_numpy(joint_rows(c["data"], dims)))
eng.init_params(0)
for i in range(3):
    eng.update(i, idx=torch.from_numpy(c["idx"][i]))
eng.update_round()
eng.synchronize()
segs = torch.cuda.memory_snapshot()
print(json.dumps({"stats_finite": bool(all(np.isfinite(eng.stats(i)).all() for i in range(3))),
                  "alloc_conf": os.environ.get("PYTORCH_HIP_ALLOC_CONF", ""),
                  "expandable_segments": sum(1 for g in segs if g.get("is_expandable")),
                  "segments": len(segs)}))
"""


def test_expandable_segments_accepted():
    """PyTorch's expandable segments map device memory with hipMemCreate /
    hipMemMap: the ABI's pointer check accepts it (allocation handle of the
    handle's device) and the update trains.  This PyTorch build may not honour
    the setting (the child reports how many segments were expandable; r06q: 0);
    tests/native/abi_host_check.cpp maps virtual memory itself either way."""
    env = dict(os.environ, ROOT=ROOT, PYTORCH_HIP_ALLOC_CONF="expandable_segments:True",
               PYTORCH_CUDA_ALLOC_CONF="expandable_segments:True")
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    print(out)
    assert out["stats_finite"], out
