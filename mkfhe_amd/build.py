"""Build the in-tree libraries:
    mkfhe_amd/lib/libmkfhe_amd.so   HIP engine for gfx950 (hipcc)
    mkfhe_amd/lib/libmkfhe_keys.so  host key material (g++, include/mkfhe_keys.h)

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
HEADERS = [os.path.join(_HERE, "csrc", f) for f in ("mkacc_device.hpp", "mkacc_host_math.hpp", "mkacc_gate.hpp", "mkacc_wide.hpp", "mkacc_widefp.hpp")] + [
    os.path.join(ROOT, "include", "mkfhe_amd.h")]
OUT = os.path.join(_HERE, "lib", "libmkfhe_amd.so")
KEYS_SOURCES = [os.path.join(_HERE, "csrc", "mkkeys.cpp")]
KEYS_HEADERS = [os.path.join(_HERE, "csrc", "mkacc_host_math.hpp"), os.path.join(ROOT, "include", "mkfhe_keys.h"),
                os.path.join(ROOT, "include", "mkfhe_amd.h")]
KEYS_OUT = os.path.join(_HERE, "lib", "libmkfhe_keys.so")
ARCH = os.environ.get("MKFHE_OFFLOAD_ARCH", "gfx950")


def _stale(out, deps) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(f) > t for f in deps)


def build_keys(force: bool = False, verbose: bool = False) -> str:
    """Host key-material library (plain C++, no GPU)."""
    if not force and not _stale(KEYS_OUT, KEYS_SOURCES + KEYS_HEADERS):
        return KEYS_OUT
    os.makedirs(os.path.dirname(KEYS_OUT), exist_ok=True)
    cxx = os.environ.get("CXX", "g++")
    # inline helpers stay private to each library (both include mkacc_host_math.hpp)
    cmd = [cxx, "-O3", "-march=x86-64-v3", "-std=c++17", "-fPIC", "-shared", "-pthread",
           "-fvisibility-inlines-hidden", "-Wl,-Bsymbolic",
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(_HERE, "csrc"),
           "-o", KEYS_OUT + ".tmp"] + KEYS_SOURCES
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(KEYS_OUT + ".tmp", KEYS_OUT)
    return KEYS_OUT


def build(force: bool = False, verbose: bool = False) -> str:
    build_keys(force, verbose)
    if not force and not _stale(OUT, SOURCES + HEADERS):
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-fvisibility-inlines-hidden", "-Wl,-Bsymbolic",
           "-Wno-unused-result", "-Wno-pass-failed", "-I", os.path.join(ROOT, "include"),
           "-Rpass-analysis=kernel-resource-usage", "-o", OUT + ".tmp"] + SOURCES
    if verbose:
        print(" ".join(cmd))
    # per-kernel VGPR / spill / occupancy report next to the library
    with open(os.path.join(os.path.dirname(OUT), "resource_usage.txt"), "w") as rep:
        subprocess.check_call(cmd, stderr=rep)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
