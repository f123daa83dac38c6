#!/usr/bin/env python3
"""Build guard: no kernel of the library may use scratch (private segment)
except the general critic kernels, whose register spills are known.

A private array the compiler could not keep in registers (e.g. a loop over it
that stayed rolled) lands in scratch: slow, and a 1024-thread optimizer launch
with 336 B of scratch per lane faulted the GPU inside the captured train-step
graph.  The allowed kernels never wait on another workgroup; the optimizer
launches do (norm handshake, xGMI exchange), and waves that need scratch are
dispatched only while the queue's scratch slots last, so a spinning grid with
scratch may not be co-resident.  mdp_create re-checks the spinning kernels at
run time (mdp_spin_kernels_scratch) and disables the spinning launches if any
has a private segment.  Run by the Makefile after the link:

    python3 tools/check_scratch.py maddpg_amd/libmaddpg_hip.so
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
# kernels allowed to spill (mangled-name prefixes)
ALLOWED = ("_Z13k_critic_gradILi", "_Z11k_grad_pairILi")  # the general critic step and the pair launch holding it


def kernel_scratch(lib):
    """{kernel: private_segment_fixed_size} over every gfx950 code object of lib."""
    out = {}
    with tempfile.TemporaryDirectory() as d:
        so = os.path.join(d, "lib.so")
        shutil.copy(lib, so)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", so], cwd=d, check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        for f in sorted(os.listdir(d)):
            if not f.endswith("gfx950"):
                continue
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", os.path.join(d, f)], check=True,
                                   capture_output=True, text=True).stdout
            name = None
            for line in notes.splitlines():
                m = re.match(r"\s+\.name:\s+(\S+)", line)
                if m:
                    name = m.group(1)
                m = re.match(r"\s+\.private_segment_fixed_size:\s+(\d+)", line)
                if m and name:
                    out[name] = max(out.get(name, 0), int(m.group(1)))
                    name = None
    return out


def main():
    lib = sys.argv[1]
    if not os.path.exists(f"{LLVM}/llvm-readelf"):
        print("check_scratch: llvm tools absent, skipped")
        return 0
    sc = kernel_scratch(lib)
    if not sc:
        print(f"check_scratch: no kernel metadata found in {lib}", file=sys.stderr)
        return 1
    bad = {k: v for k, v in sc.items() if v and not k.startswith(ALLOWED)}
    if bad:
        for k, v in sorted(bad.items()):
            print(f"check_scratch: {k} uses {v} B of scratch per lane", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
