#!/usr/bin/env python3
"""Average per-dispatch PMC values of one kernel across rocprofv3 counter CSVs.
usage: pmc_summary.py DIR [KERNEL_SUBSTRING]"""
import collections, csv, glob, re, sys
d = sys.argv[1]; pat = sys.argv[2] if len(sys.argv) > 2 else "mk_step_kernel"
agg = collections.defaultdict(float); cnt = collections.Counter()
for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        # the later steps only: skip the FIRST instantiation (<DG, METHOD, true, ...>)
        if pat not in r["Kernel_Name"] or re.search(r"<(\d+, )+true", r["Kernel_Name"]):
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
for k in sorted(agg):
    print(f"{k:28s} {agg[k] / cnt[k]:16.1f}  (n={cnt[k]})")

if len(sys.argv) > 3:
    # sys.argv[3] = paramset: write the per-launch HBM traffic record bench.py reads
    import json
    f, w = agg.get("FETCH_SIZE"), agg.get("WRITE_SIZE")
    if f is not None and w is not None:
        f /= cnt["FETCH_SIZE"]; w /= cnt["WRITE_SIZE"]
        rec = {"paramset": sys.argv[3], "kernel": pat, "fetch_size_kb": f, "write_size_kb": w,
               "traffic_bytes": (2 * f + w) * 1024,
               "correction": "MI355X_MICROARCH.md HBM: FETCH_SIZE (KB) x2 for 16-B/lane coalesced reads on gfx950, "
                             "WRITE_SIZE (KB) x1; separate --pmc passes; per dispatch of the step kernel",
               "source": d}
        out = f"profiles/traffic_{sys.argv[3]}.json"
        json.dump(rec, open(out, "w"), indent=1)
        print("wrote", out, rec["traffic_bytes"])
