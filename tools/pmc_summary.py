#!/usr/bin/env python3
"""Average per-dispatch PMC values of one kernel across rocprofv3 counter CSVs.

usage: pmc_summary.py DIR [KERNEL_SUBSTRING [PARAMSET]]

With PARAMSET, writes profiles/traffic_<PARAMSET>.json, the per-launch HBM
traffic record bench.py reports as roofline.traffic: FETCH_SIZE and WRITE_SIZE
from separate --pmc passes, corrected as MI355X_MICROARCH.md prescribes, and
stamped with the identity of what was measured -- the kernel's full name, the
isa id of its machine code in the library that ran (tools/kernel_isa.py,
mkfhe_amd/lib/libmkfhe_amd.kernel_isa.json) and the library's build info.
bench.py uses the record only while the benched library's kernel has that isa
id."""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> int:
    d = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "mk_step_kernel"
    agg = collections.defaultdict(float)
    cnt = collections.Counter()
    names = collections.Counter()
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            # the later steps only: skip the FIRST instantiation (<DG, METHOD, true, ...>)
            if pat not in r["Kernel_Name"] or re.search(r"<(\d+, )+true", r["Kernel_Name"]):
                continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[r["Counter_Name"]] += 1
            names[r["Kernel_Name"]] += 1
    for k in sorted(agg):
        print(f"{k:28s} {agg[k] / cnt[k]:16.1f}  (n={cnt[k]})")
    for n, c in names.items():
        print(f"kernel: {n} ({c} rows)")

    if len(sys.argv) > 3:
        f, w = agg.get("FETCH_SIZE"), agg.get("WRITE_SIZE")
        if f is None or w is None:
            print("no FETCH_SIZE / WRITE_SIZE pass: no traffic record written")
            return 1
        if len(names) != 1:
            print(f"expected one kernel instantiation, found {len(names)}: no traffic record written")
            return 1
        sym = next(iter(names))
        sys.path.insert(0, ROOT)
        from mkfhe_amd import _lib
        ids = json.load(open(_lib.LIB_PATH[:-3] + ".kernel_isa.json"))
        f /= cnt["FETCH_SIZE"]
        w /= cnt["WRITE_SIZE"]
        rec = {"paramset": sys.argv[3], "kernel": pat, "kernel_symbol": sym, "kernel_isa": ids.get(sym),
               "build_info": _lib.load().build_info,
               "fetch_size_kb": f, "write_size_kb": w, "traffic_bytes": (2 * f + w) * 1024,
               "correction": "MI355X_MICROARCH.md HBM: FETCH_SIZE (KB) x2 for 16-B/lane coalesced reads on gfx950, "
                             "WRITE_SIZE (KB) x1; separate --pmc passes; per dispatch of the step kernel",
               "launch": "MKACC_STREAMS=1 during the passes: one dispatch is one step of the whole batch "
                         "(tools/gpu_lib.sh pmc), the bench's bytes_per_launch",
               "source": d}
        out = os.path.join(ROOT, "profiles", f"traffic_{sys.argv[3]}.json")
        json.dump(rec, open(out, "w"), indent=1)
        print("wrote", out, rec["traffic_bytes"], rec["kernel_isa"])
    return 0


if __name__ == "__main__":
    sys.exit(main())
