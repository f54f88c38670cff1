"""Build the in-tree HIP engine: mkfhe_amd/lib/libmkfhe_amd.so (gfx950).

    python -m mkfhe_amd.build [--force]

Plain hipcc invocation -- no JIT cache, so the .so travels with the repo
snapshot to the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(_HERE)
SOURCES = [os.path.join(_HERE, "csrc", "mkacc_engine.hip")]
HEADERS = [os.path.join(_HERE, "csrc", f) for f in ("mkacc_device.hpp", "mkacc_host_math.hpp", "mkacc_gate.hpp")] + [
    os.path.join(ROOT, "include", "mkfhe_amd.h")]
OUT = os.path.join(_HERE, "lib", "libmkfhe_amd.so")
ARCH = os.environ.get("MKFHE_OFFLOAD_ARCH", "gfx950")


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(f) > t for f in SOURCES + HEADERS)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-result", "-Wno-pass-failed", "-I", os.path.join(ROOT, "include"),
           "-o", OUT + ".tmp"] + SOURCES
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
