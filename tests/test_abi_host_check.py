"""The C ABI under host AddressSanitizer + UBSan (the reference
has no sanitizer or NaN check, `tf_util.py:322`).

tests/native/abi_host_check links the C-ABI shim (maddpg_amd/csrc/mdp_api.cpp)
built with -fsanitize=address,undefined on the host side against the shipped
kernel objects and calls every entry point of include/maddpg_hip.h:
* `cpu` (no GPU): config validation (every rule of build_layout), arena
  layout, the co-residency plan, and every entry point on a NULL handle and on
  a handle whose mdp_create failed -- each must return < 0 without touching
  device memory;
* `gpu` (device 0): three configurations (register H=64 kernels, general
  H=128 kernels with 6 agents, a ragged DDPG case) through the whole lifecycle
  -- parameters, RNG state, env steps, strict / throughput rounds, graphs,
  profiling, every refused call on a live handle, destroy.
A sanitizer report aborts the binary (non-zero exit), so "OK" means none fired.
LeakSanitizer runs in the CPU mode only: its exit-time scan hangs the GPU-mode
binary when the parent process (this pytest run) holds a HIP context, while
the same binary run alone is leak-free apart from the ROCm runtime's own
allocations (profiles/r05m_host_sanitizers.log: run A leak check on, run C
with a parent context and the leak check off, run B both -- hung at exit).
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "native", "abi_host_check")
ENV = dict(os.environ, ASAN_OPTIONS="verify_asan_link_order=0:detect_leaks=1:abort_on_error=0",
           UBSAN_OPTIONS="print_stacktrace=1",
           LSAN_OPTIONS="suppressions=" + os.path.join(ROOT, "tests", "native", "lsan.supp"))


def _binary():
    if shutil.which("hipcc") or os.path.exists("/opt/rocm/bin/hipcc"):
        subprocess.run(["make", "-C", os.path.join(ROOT, "maddpg_amd", "csrc"), "-j8", "host-check"],
                       check=True, capture_output=True, timeout=900)
    if not os.path.exists(BIN):
        pytest.skip("abi_host_check not built (no hipcc here)")
    return BIN


def _run(mode, timeout):
    p = subprocess.run([_binary(), mode], capture_output=True, text=True, timeout=timeout, env=ENV, cwd="/tmp")
    out = p.stdout + p.stderr
    print(out[-4000:])
    assert p.returncode == 0, out[-4000:]
    assert "OK " in p.stdout and "ERROR: AddressSanitizer" not in out and "runtime error" not in out


def test_abi_host_sanitizers_cpu():
    _run("cpu", 300)


@pytest.mark.gpu
def test_abi_host_sanitizers_gpu():
    if not os.path.exists(BIN):
        pytest.fail("tests/native/abi_host_check missing: run __graft_entry__.build() first")
    env = dict(ENV, ASAN_OPTIONS="verify_asan_link_order=0:detect_leaks=0:abort_on_error=0")
    p = subprocess.run([BIN, "gpu"], capture_output=True, text=True, timeout=300, env=env, cwd="/tmp")
    out = p.stdout + p.stderr
    print(out[-6000:])
    assert p.returncode == 0, out[-6000:]
    assert "OK " in p.stdout and "ERROR: AddressSanitizer" not in out and "runtime error" not in out
