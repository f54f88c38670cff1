#!/usr/bin/env python3
"""Per-kernel machine-code identity of a built engine library.

    kernel_isa.py LIB.so [OUT.json]          write {demangled kernel name: isa id}
    kernel_isa.py --diff OLD.json NEW.json   kernels whose machine code changed

The isa id of a kernel is the SHA-256 prefix of its gfx950 disassembly with the
addresses and raw encodings stripped (branch operands are relative, so the text
does not depend on where the linker put the function).  Two builds whose ids
match for a kernel run the same instructions for it: a performance or HBM
traffic record taken of one applies to the other.  mkfhe_amd/build.py writes
mkfhe_amd/lib/kernel_isa.json next to every library; the traffic records under
profiles/ carry the id of the kernel they measured and bench.py only reports a
record whose id matches the library it runs.

A kernel name that occurs in several translation units (the small helper
kernels each unit instantiates) maps to the sorted, '+'-joined ids."""
from __future__ import annotations

import hashlib
import json
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from isa_audit import disassemble  # noqa: E402

_SYM = re.compile(r"^[0-9a-f]+ <(.+)>:$")


def split_functions(text: str) -> list[tuple[str, str]]:
    """(mangled symbol, normalised instruction text) of every function."""
    out, name, body = [], None, []
    for raw in text.splitlines():
        s = raw.strip()
        m = _SYM.match(s)
        if m:
            if name is not None:
                out.append((name, "\n".join(body)))
            name, body = m.group(1), []
            continue
        # (objdump's per-file header lines -- "<tmp path>: file format elf64-amdgpu" --
        # separate the code objects of the units and belong to no function)
        if name is None or not s or s.startswith(("Disassembly", ";")) or "file format" in s:
            continue
        s = s.split("//")[0].strip()
        if s:
            body.append(" ".join(s.split()))
    if name is not None:
        out.append((name, "\n".join(body)))
    return out


def demangle(names: list[str]) -> list[str]:
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True)
    out = r.stdout.splitlines()
    return out if len(out) == len(names) else names


def kernel_ids(lib: str) -> dict[str, str]:
    funcs = split_functions(disassemble(lib))
    names = demangle([f[0] for f in funcs])
    ids: dict[str, set[str]] = {}
    for dn, (_, body) in zip(names, funcs):
        ids.setdefault(dn, set()).add(hashlib.sha256(body.encode()).hexdigest()[:16])
    return {k: "+".join(sorted(v)) for k, v in sorted(ids.items())}


def main() -> int:
    if sys.argv[1] == "--diff":
        a, b = json.load(open(sys.argv[2])), json.load(open(sys.argv[3]))
        same = [k for k in a if k in b and a[k] == b[k]]
        changed = [k for k in a if k in b and a[k] != b[k]]
        print(f"{len(same)} kernels identical, {len(changed)} changed, "
              f"{len(set(a) - set(b))} only in {sys.argv[2]}, {len(set(b) - set(a))} only in {sys.argv[3]}")
        for k in changed:
            print("CHANGED", k)
        return 1 if changed else 0
    ids = kernel_ids(sys.argv[1])
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(ids, f, indent=1)
    else:
        print(json.dumps(ids, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
