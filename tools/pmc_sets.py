#!/usr/bin/env python3
"""Summarise the SQ/TCC counter passes of one configuration (tools/gpu_lib.sh pmcset).

    pmc_sets.py DIR KERNEL_SUBSTRING GATES [STEPS_PER_GATE_STEP]

DIR holds one sub-directory per pass (sq1, sq2, l2) with rocprofv3's
run_counter_collection.csv.  Every pass runs the bench with MKACC_STREAMS=1 and a
short LWE dimension, so every dispatch of the step kernel is one accumulator step
of the whole batch (GATES gates).  Prints the per-dispatch means of every counter
of the step kernel and the derived figures DESIGN.md quotes: VALU instructions
per gate-step, waves, VALU-active and waiting fractions of the wave cycles, LDS
bank-conflict cycles per LDS instruction, and the L2 hit rate."""
from __future__ import annotations

import csv
import glob
import os
import sys
from collections import defaultdict


def load(dirname: str, kern: str) -> dict[str, float]:
    sums: dict[str, float] = defaultdict(float)
    counts: dict[str, int] = defaultdict(int)
    for f in sorted(glob.glob(os.path.join(dirname, "*", "run_counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            if kern not in row["Kernel_Name"]:
                continue
            sums[row["Counter_Name"]] += float(row["Counter_Value"])
            counts[row["Counter_Name"]] += 1
    return {k: sums[k] / counts[k] for k in sums}


def main() -> int:
    d, kern, gates = sys.argv[1], sys.argv[2], int(sys.argv[3])
    c = load(d, kern)
    if not c:
        print("no dispatch of", kern)
        return 1
    for k in sorted(c):
        print(f"{k:34s} {c[k]:16.1f}")
    out = {}
    if "SQ_INSTS_VALU" in c:
        out["VALU instructions per gate-step"] = c["SQ_INSTS_VALU"] / gates
    if "SQ_INSTS_LDS" in c:
        out["LDS instructions per gate-step"] = c["SQ_INSTS_LDS"] / gates
    if "SQ_INSTS_VMEM_RD" in c:
        out["VMEM reads per gate-step"] = c["SQ_INSTS_VMEM_RD"] / gates
    if "SQ_WAVE_CYCLES" in c:
        wc = c["SQ_WAVE_CYCLES"]
        for n in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_LDS"):
            if n in c:
                out[f"{n} / SQ_WAVE_CYCLES"] = c[n] / wc
    if "SQ_LDS_BANK_CONFLICT" in c and "SQ_INSTS_LDS" in c and c["SQ_INSTS_LDS"]:
        out["LDS bank-conflict cycles per LDS instruction"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_INSTS_LDS"]
    h = c.get("TCC_HIT_sum")
    m = c.get("TCC_MISS_sum")
    if h is not None and m is not None and h + m:
        out["L2 hit rate"] = h / (h + m)
    print()
    for k, v in out.items():
        print(f"{k:46s} {v:10.4f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
