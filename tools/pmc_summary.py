#!/usr/bin/env python3
"""Average per-dispatch PMC values of one kernel across rocprofv3 counter CSVs.
usage: pmc_summary.py DIR [KERNEL_SUBSTRING]"""
import collections, csv, glob, sys
d = sys.argv[1]; pat = sys.argv[2] if len(sys.argv) > 2 else "mk_step_kernel"
agg = collections.defaultdict(float); cnt = collections.Counter()
for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"] or "true" in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
for k in sorted(agg):
    print(f"{k:28s} {agg[k] / cnt[k]:16.1f}  (n={cnt[k]})")
