#!/usr/bin/env python3
"""ISA audit of a built engine library: every store of more than 8 bytes must
keep its data VGPRs unwritten for 2 wait states after it issues (gfx950 VMEM
store-data hazard; see bstore4 in mkfhe_amd/csrc/mkacc_device.hpp).  hipcc does
not pad buffer stores that use an SGPR soffset, and a violation silently
corrupts part of the stored data under load.

usage: isa_audit.py LIB.so [--verbose]     exit status 1 on any violation

The gfx950 code object is unbundled from the library's .hip_fatbin section
(llvm-objcopy + clang-offload-bundler) and disassembled with llvm-objdump."""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
WAIT_STATES = 2
# second check: a v_mad_u64_u32 writing its carry-out to VCC (the pinned inline-asm
# multiply-adds of mkacc_device.hpp) must be followed by VCC_WAIT wait states before
# any SALU instruction that writes or reads VCC, or an s_cbranch_vcc*.  hipcc does not
# count an asm statement as a VALU write of VCC, and a late VALU write of VCC that
# lands after the SALU's own write sent every wave of mk_lat_kernel down the
# index-party path (intermittent wrong accumulators).
VCC_WAIT = 8

_STORE = re.compile(r"^(buffer|global|flat|scratch)_store_(dwordx3|dwordx4|b96|b128)\b")
_VRANGE = re.compile(r"v\[(\d+):(\d+)\]|v(\d+)\b")


def disassemble(lib: str) -> str:
    """Disassembly of every gfx950 code object in the library: a library linked
    from several translation units holds one offload bundle per unit,
    concatenated in .hip_fatbin (each starts with the bundle magic)."""
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    out = []
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fat])
        blob = open(fat, "rb").read()
        starts, i = [], blob.find(magic)
        while i >= 0:
            starts.append(i)
            i = blob.find(magic, i + 1)
        if not starts:
            raise RuntimeError(f"{lib}: no offload bundle in .hip_fatbin")
        for n, s in enumerate(starts):
            e = starts[n + 1] if n + 1 < len(starts) else len(blob)
            part, obj = os.path.join(d, f"b{n}.bin"), os.path.join(d, f"b{n}.o")
            with open(part, "wb") as f:
                f.write(blob[s:e])
            subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--type=o", "--unbundle", f"--input={part}",
                                   f"--output={obj}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"])
            out.append(subprocess.check_output([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", obj], text=True))
    return "\n".join(out)


def vregs(operand: str) -> set[int]:
    m = _VRANGE.match(operand.strip())
    if not m:
        return set()
    if m.group(3) is not None:
        return {int(m.group(3))}
    return set(range(int(m.group(1)), int(m.group(2)) + 1))


def writes_vgprs(mnem: str, ops: list[str]) -> set[int]:
    if not ops:
        return set()
    if mnem.startswith(("v_cmp", "v_readlane", "v_readfirstlane")):
        return set()
    if mnem.startswith("v_") or mnem.startswith(("buffer_load", "global_load", "flat_load", "scratch_load",
                                                   "ds_read", "ds_load")):
        return vregs(ops[0])
    return set()


def audit(text: str, verbose: bool = False):
    kernel, insts, violations, stores = None, [], [], 0
    vcc_sites = 0

    def flush():
        nonlocal stores, vcc_sites
        for i, (mn, ops, line) in enumerate(insts):
            if mn == "v_mad_u64_u32" and len(ops) > 1 and ops[1] == "vcc":
                ws = 0
                for mn2, ops2, line2 in insts[i + 1:]:
                    if ws >= VCC_WAIT:
                        break
                    if mn2 == "s_nop":
                        ws += int(ops2[0], 0) + 1 if ops2 else 1
                        continue
                    if (mn2.startswith("s_cbranch_vcc") or
                            (mn2.startswith("s_") and any(o in ("vcc", "vcc_lo", "vcc_hi") for o in ops2))):
                        vcc_sites += 1
                        violations.append((kernel, line.strip(), line2.strip()))
                        break
                    ws += 1
            if not _STORE.match(mn):
                continue
            stores += 1
            data = vregs(ops[0] if mn.startswith("buffer") else ops[1])
            ws = 0
            for mn2, ops2, line2 in insts[i + 1:]:
                if ws >= WAIT_STATES:
                    break
                if mn2 == "s_nop":
                    ws += int(ops2[0], 0) + 1 if ops2 else 1
                    continue
                if mn2.startswith("s_waitcnt") and "vmcnt(0)" in line2:
                    break
                if writes_vgprs(mn2, ops2) & data:
                    violations.append((kernel, line.strip(), line2.strip()))
                    break
                ws += 1

    for raw in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", raw.strip())
        if m:
            flush()
            kernel, insts = m.group(1), []
            continue
        s = raw.strip()
        if not s or s.startswith(("Disassembly", ";")) or kernel is None:
            continue
        s = s.split("//")[0].strip()
        if not s:
            continue
        parts = s.split(None, 1)
        mn = parts[0]
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        insts.append((mn, ops, s))
    flush()
    return stores, violations, vcc_sites


def main() -> int:
    lib = sys.argv[1]
    stores, bad, vcc = audit(disassemble(lib), "--verbose" in sys.argv)
    for k, st, wr in bad[:20]:
        print(f"VIOLATION in {k}:\n    {st}\n    {wr}")
    print(f"{os.path.basename(lib)}: {stores} stores of more than 8 bytes, {len(bad) - vcc} data-register hazards, "
          f"{vcc} VCC carry-out hazards")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
