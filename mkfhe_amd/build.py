"""Build the in-tree libraries:
    mkfhe_amd/lib/libmkfhe_amd.so   HIP engine for gfx950 (hipcc)
    mkfhe_amd/lib/libmkfhe_keys.so  host key material (g++, include/mkfhe_keys.h)

    python -m mkfhe_amd.build [--force]
    python -m mkfhe_amd.build --variant NAME [-DFLAG ...]   # A/B engine build -> lib/variants/NAME.so

Plain hipcc invocation -- no JIT cache, so the .so travels with the repo
snapshot to the GPU box.

Every library carries its build identity (mkacc_build_info / mkkg_build_info):
the SHA-256 prefix of its public header and of all of its sources, and the
extra compile flags.  The Python loaders (_lib.load, keys.load) refuse a
library whose ABI version or header id differs from the tree they run in, and
the default libraries must also match the sources (a stale build is refused).
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(_HERE)
SOURCES = [os.path.join(_HERE, "csrc", f) for f in ("mkacc_engine.hip", "mkacc_steps.hip")]
HEADERS = [os.path.join(_HERE, "csrc", f) for f in ("mkacc_kernels.hpp", "mkacc_step2.hpp", "mkacc_quad.hpp",
                                                    "mkacc_device.hpp", "mkacc_host_math.hpp",
                                                    "mkacc_gate.hpp", "mkacc_wide.hpp", "mkacc_fp64.hpp",
                                                    "mkacc_widereg2.hpp", "mkacc_layout2.hpp")] + [
    os.path.join(ROOT, "include", "mkfhe_amd.h")]
OUT = os.path.join(_HERE, "lib", "libmkfhe_amd.so")
KEYS_SOURCES = [os.path.join(_HERE, "csrc", "mkkeys.cpp")]
KEYS_HEADERS = [os.path.join(_HERE, "csrc", "mkacc_host_math.hpp"), os.path.join(ROOT, "include", "mkfhe_keys.h"),
                os.path.join(ROOT, "include", "mkfhe_amd.h")]
KEYS_OUT = os.path.join(_HERE, "lib", "libmkfhe_keys.so")
ARCH = os.environ.get("MKFHE_OFFLOAD_ARCH", "gfx950")
ENGINE_HEADER = os.path.join(ROOT, "include", "mkfhe_amd.h")
KEYS_HEADER = os.path.join(ROOT, "include", "mkfhe_keys.h")


def file_id(paths) -> str:
    """SHA-256 prefix (16 hex digits) of the concatenated file contents."""
    h = hashlib.sha256()
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def engine_ids() -> dict:
    # this file holds the per-unit compile flags (STEP2_SCHED, UNITS), so it is
    # part of the source identity: a library built with other flags is stale
    return {"header": file_id([ENGINE_HEADER]), "source": file_id(SOURCES + HEADERS + [os.path.abspath(__file__)])}


def keys_ids() -> dict:
    return {"header": file_id([KEYS_HEADER, ENGINE_HEADER]), "source": file_id(KEYS_SOURCES + KEYS_HEADERS)}


def _id_defines(prefix: str, ids: dict, flags: list[str]) -> list[str]:
    return [f'-D{prefix}_HEADER_ID="{ids["header"]}"', f'-D{prefix}_SOURCE_ID="{ids["source"]}"',
            f'-D{prefix}_BUILD_FLAGS="{" ".join(flags)}"']


def _stale(out, deps) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(f) > t for f in deps)


# AddressSanitizer + UBSan build of the key library (tests/test_sanitize.py loads it
# through MKFHE_KEYS_LIB with libasan preloaded): lib/variants/libmkfhe_keys_asan.so
SANITIZE = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"]
KEYS_ASAN_OUT = os.path.join(_HERE, "lib", "variants", "libmkfhe_keys_asan.so")


def build_keys(force: bool = False, verbose: bool = False, sanitize: bool = False) -> str:
    """Host key-material library (plain C++, no GPU); sanitize: the ASan/UBSan build."""
    out = KEYS_ASAN_OUT if sanitize else KEYS_OUT
    if not force and not _stale(out, KEYS_SOURCES + KEYS_HEADERS):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cxx = os.environ.get("CXX", "g++")
    opt = SANITIZE if sanitize else ["-O3"]
    # inline helpers stay private to each library (both include mkacc_host_math.hpp)
    cmd = [cxx, *opt, "-march=x86-64-v3", "-std=c++17", "-fPIC", "-shared", "-pthread",
           "-fvisibility-inlines-hidden", "-Wl,-Bsymbolic",
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(_HERE, "csrc"),
           *_id_defines("MKKG", keys_ids(), ["sanitize"] if sanitize else []), "-o", out + ".tmp"] + KEYS_SOURCES
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    return out


# Machine-scheduler strategy of the step2 unit at dg = 3 (the headline kernel):
# max-memory-clause schedules it at 256 VGPRs with no spills (the default
# strategy spills 6) and ran 154.6-155.3 us per STD128_MKNTRU launch against
# 159.0-159.9 (profiles/r3/ab_sched.txt); the ISA audit stays clean with it.
STEP2_SCHED = {3: ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"]}
# Shoup products of the transforms written in C (MKACC_BFLY_C, mkacc_device.hpp):
# no s_nop per butterfly; -1.7 to -2.1 % per headline step, +0.6 % for mk_step_kernel
# at dg = 4 (profiles/r5/ab_hl_bfly_c.txt), so only the later-step units of
# mk_step2_kernel take it (dg = 2: -0.3 to -0.5 % per config-3 step,
# profiles/r5/ab_c3_bfly_c.txt; its first-step kernels, a unit of their own,
# would spill at dg = 3).
STEP2_BFLY = {2: ["-DMKACC_BFLY_C=1"], 3: ["-DMKACC_BFLY_C=1"]}
# and mk_lat_kernel (small batches, few waves per SIMD to hide a wait state): a
# 64-gate STD128_MKNTRU batch 65.7 -> 63.0 ms (profiles/r5/ab_lat_bfly_c.txt)
LAT_BFLY = ["-DMKACC_BFLY_C=1"]
# and mk_quad_kernel (one wave per SIMD: the asm form's wait states are not hidden)
QUAD_BFLY = ["-DMKACC_BFLY_C=1"]
# mk_step_kernel at dg = 4 (config 4): the forward transforms only (MKACC_BFLY_C=2);
# in every transform it needs 8 B of scratch and is 0.6 % slower, forward-only is
# spill-free and 1.0-1.1 % faster (profiles/r5/ab_c4_bfly_c.txt)
STEP_BFLY = {4: ["-DMKACC_BFLY_C=2"]}

# Translation units of the engine library, compiled in parallel and linked into
# one .so: the host unit (C ABI, batch / gate / primitive kernels) and the step
# kernel units of mkacc_steps.hip (one per digit count and kernel kind, and the
# two 64-bit word paths), which the host unit launches through mkacc_tu.  Only the
# kernels the engine selects are built: mk_step2_kernel at dg <= 3, mk_step_kernel
# at dg >= 4, mk_lat_kernel for small batches, the FP64 register-resident kernel
# below 2^50 and the integer 64-bit kernel above (round 5 retired the variants that
# lost their A/B runs; DESIGN.md s7 keeps their records).
UNITS = [("engine", "mkacc_engine.hip", [])] + [
    (f"step_dg{d}", "mkacc_steps.hip", [f"-DMKACC_TU_DG={d}", "-DMKACC_TU_PART=0"] + STEP_BFLY.get(d, []))
    for d in (4, 5)] + [
    (f"lat_dg{d}", "mkacc_steps.hip", [f"-DMKACC_TU_DG={d}", "-DMKACC_TU_PART=1"] + LAT_BFLY) for d in (2, 3, 4)] + [
    (f"step2_dg{d}", "mkacc_steps.hip", [f"-DMKACC_TU_DG={d}", "-DMKACC_TU_PART=2"] + STEP2_SCHED.get(d, []) +
     STEP2_BFLY.get(d, []))
    for d in (2, 3)] + [
    (f"step2f_dg{d}", "mkacc_steps.hip", [f"-DMKACC_TU_DG={d}", "-DMKACC_TU_PART=3"] + STEP2_SCHED.get(d, []))
    for d in (2, 3)] + [
    (f"quad_dg{d}", "mkacc_steps.hip", [f"-DMKACC_TU_DG={d}", "-DMKACC_TU_PART=4"] + QUAD_BFLY) for d in (2, 3, 4, 5)] + [
    ("wide", "mkacc_steps.hip", ["-DMKACC_TU_WIDE=1"]), ("widereg2", "mkacc_steps.hip", ["-DMKACC_TU_WIDE=2"])]


def _jobs() -> int:
    for var in ("MAX_JOBS", "MKFHE_BUILD_JOBS"):
        if os.environ.get(var, "").isdigit():
            return max(1, int(os.environ[var]))
    return max(1, min(len(UNITS), os.cpu_count() or 1))


def included_files(path: str, seen=None) -> list[str]:
    """path and every in-tree header it reaches through #include "..." (transitively)."""
    import re
    seen = [] if seen is None else seen
    path = os.path.normpath(path)
    if path in seen or not os.path.exists(path):
        return seen
    seen.append(path)
    with open(path) as f:
        for m in re.finditer(r'^\s*#\s*include\s+"([^"]+)"', f.read(), re.M):
            included_files(os.path.join(os.path.dirname(path), m.group(1)), seen)
    return seen


_COMPILER_ID: dict[str, str] = {}


def compiler_id(hipcc: str) -> str:
    """The toolchain a unit object was built with: `hipcc --version` (ROCm and clang
    versions) plus the resolved path and mtime of the compiler binary, so a cached
    object is never linked next to units from another toolchain."""
    if hipcc not in _COMPILER_ID:
        r = subprocess.run([hipcc, "--version"], capture_output=True, text=True)
        real = os.path.realpath(hipcc)
        st = os.stat(real) if os.path.exists(real) else None
        _COMPILER_ID[hipcc] = f"{r.stdout}|{real}|{st.st_mtime_ns if st else 0}"
    return _COMPILER_ID[hipcc]


def unit_key(path: str, cmd: list[str]) -> str:
    """Identity of one translation unit's compile: its sources, its command line and
    the compiler (compiler_id)."""
    h = hashlib.sha256(" ".join(cmd).encode())
    h.update(compiler_id(cmd[0]).encode())
    for f in included_files(path):
        with open(f, "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()


def compile_engine(out: str, flags: list[str], report: str, verbose: bool = False, only=None) -> str:
    """hipcc the engine units into `out` with extra `flags` (-D switches of A/B builds).
    only: names of the units to compile with the flags; the others are linked from
    the default build's objects (an A/B variant of one kernel family)."""
    from concurrent.futures import ThreadPoolExecutor

    os.makedirs(os.path.dirname(out), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    objdir = out[:-3] + ".objs"
    os.makedirs(objdir, exist_ok=True)
    common = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
              "-fvisibility-inlines-hidden", "-Wno-unused-result", "-Wno-pass-failed",
              "-I", os.path.join(ROOT, "include"), *_id_defines("MKACC", engine_ids(), flags), *flags,
              "-Rpass-analysis=kernel-resource-usage"]

    ids_flags = _id_defines("MKACC", engine_ids(), flags)

    def unit(u):
        name, src, defs = u
        obj = os.path.join(objdir, name + ".o")
        path = os.path.join(_HERE, "csrc", src)
        cmd = common + defs + ["-c", "-o", obj, path]
        # a step unit whose sources (its file and the headers it reaches) and flags are
        # unchanged keeps its object: the build-id defines only reach the host unit
        key = unit_key(path, [c for c in cmd if c not in ids_flags] + (ids_flags if name == "engine" else []))
        stamp = obj + ".key"
        if os.path.exists(obj) and os.path.exists(stamp) and open(stamp).read() == key:
            rep = obj + ".res"
            return name, obj, subprocess.CompletedProcess(cmd, 0, "", open(rep).read() if os.path.exists(rep) else "")
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode == 0:
            with open(obj + ".res", "w") as f:
                f.write(r.stderr)
            with open(stamp, "w") as f:
                f.write(key)
        elif os.path.exists(stamp):
            os.remove(stamp)
        return name, obj, r

    # a variant always recompiles the host unit too: it carries the build
    # identity (mkacc_build_info's flags) and the host-side A/B switches
    if only is not None:
        only = set(only) | {"engine"}
    units = UNITS if only is None else [u for u in UNITS if u[0] in only]
    with ThreadPoolExecutor(max_workers=_jobs()) as ex:
        results = list(ex.map(unit, units))
    if only is not None:
        base = OUT[:-3] + ".objs"
        results += [(u[0], os.path.join(base, u[0] + ".o"), subprocess.CompletedProcess([], 0, "", ""))
                    for u in UNITS if u[0] not in only]
    # per-kernel VGPR / spill / occupancy report next to the library
    with open(report, "w") as rep:
        for name, _, r in results:
            rep.write(f"### unit {name}\n{r.stderr}")
    for name, _, r in results:
        if r.returncode != 0:
            raise subprocess.CalledProcessError(r.returncode, f"hipcc unit {name}", r.stdout, r.stderr[-4000:])
    link = [hipcc, f"--offload-arch={ARCH}", "--hip-link", "-shared", "-fPIC", "-Wl,-Bsymbolic", "-o", out + ".tmp"] + [
        obj for _, obj, _ in results]
    if verbose:
        print(" ".join(link), flush=True)
    subprocess.check_call(link)
    os.replace(out + ".tmp", out)
    write_kernel_ids(out)
    return out


def kernel_ids_path(lib: str) -> str:
    """The per-kernel machine-code identity file written next to a library."""
    return lib[:-3] + ".kernel_isa.json"


def write_kernel_ids(lib: str) -> str:
    """{demangled kernel: isa id} of the library (tools/kernel_isa.py): the traffic
    records under profiles/ name the id of the kernel they measured, and bench.py
    reports a record only for a library whose kernel has the same machine code."""
    import json
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import kernel_isa
    out = kernel_ids_path(lib)
    with open(out + ".tmp", "w") as f:
        json.dump(kernel_isa.kernel_ids(lib), f, indent=1)
    os.replace(out + ".tmp", out)
    return out


def build(force: bool = False, verbose: bool = False) -> str:
    build_keys(force, verbose)
    # this file holds the per-unit compile flags, so a change here rebuilds too
    if not force and not _stale(OUT, SOURCES + HEADERS + [os.path.abspath(__file__)]):
        return OUT
    return compile_engine(OUT, [], os.path.join(os.path.dirname(OUT), "resource_usage.txt"), verbose)


def build_variant(name: str, flags: list[str], verbose: bool = False, only=None) -> str:
    """An A/B build of the engine with extra -D switches: lib/variants/NAME.so
    (only: recompile just these units, the rest from the default build)."""
    if only is not None:
        build()
    out = os.path.join(_HERE, "lib", "variants", name + ".so")
    return compile_engine(out, flags, out[:-3] + ".res", verbose, only)


if __name__ == "__main__":
    if "--keys-asan" in sys.argv:
        print(build_keys(force="--force" in sys.argv, verbose=True, sanitize=True))
    elif "--variant" in sys.argv:
        args = list(sys.argv[1:])
        only = None
        if "--units" in args:
            j = args.index("--units")
            only = args[j + 1].split(",")
            del args[j:j + 2]
        i = args.index("--variant")
        print(build_variant(args[i + 1], args[i + 2:], verbose=True, only=only))
    else:
        print(build(force="--force" in sys.argv, verbose=True))
