"""Register-budget guard (CPU, no GPU).

The default-path kernels are spill-free only by a narrow margin: the dg = 3
steady `mk_step2_kernel` (the headline STD128_MKNTRU kernel) sits at exactly
256 VGPRs and stays spill-free only under the max-memory-clause machine
scheduler (the default scheduler spills 6 VGPRs there and costs
3 %).  A compiler update or a new live value would bring spills back silently,
so this test reads the per-kernel report the build writes
(`-Rpass-analysis=kernel-resource-usage` -> mkfhe_amd/lib/resource_usage.txt)
and fails if any default-path kernel spills or leaves its occupancy budget.
"""
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT

REPORT = os.path.join(ROOT, "mkfhe_amd", "lib", "resource_usage.txt")


def parse_report(text):
    """[(unit, demangled kernel name, {field: int})] from a kernel-resource-usage report."""
    rows, unit, cur = [], None, None
    for line in text.splitlines():
        if line.startswith("### unit"):
            unit = line.split()[-1]
            continue
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"unit": unit, "mangled": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+(VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|ScratchSize \[bytes/lane\]|"
                      r"Occupancy \[waves/SIMD\]): (\d+)", line)
        if m and cur is not None:
            cur[m.group(1)] = int(m.group(2))
    names = [r["mangled"] for r in rows]
    filt = shutil.which("c++filt") or shutil.which("llvm-cxxfilt")
    if filt and names:
        dem = subprocess.run([filt], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
        for r, d in zip(rows, dem):
            r["name"] = d
    for r in rows:
        r.setdefault("name", r["mangled"])
    return rows


def _rows():
    if not os.path.exists(REPORT):
        pytest.skip("engine not built here (no resource report)")
    with open(REPORT) as f:
        rows = parse_report(f.read())
    assert rows, "empty resource report"
    return rows


# (pattern on the demangled name, max VGPRs, min waves/SIMD) of every kernel the
# default build launches on the hot path; each must also have no VGPR spill and
# no scratch.  (SGPR spills are not counted: they go to VGPR lanes with
# v_writelane, not to memory, and cost a few SALU-side moves per launch.)
BUDGET = [
    (r"mk_step2_kernel<[23], [01], false>", 256, 2),     # batch step, dg <= 3 (headline: <3, 0, false>)
    (r"mk_step2_kernel<2, [01], true>", 256, 2),         # first (KDM) step at dg = 2
    (r"mk_step2_kernel<3, 1, true>", 256, 2),
    (r"mk_lat_kernel<\d, [01], (true|false)>", 256, 2),  # small-batch kernel, every digit count
    (r"mk_latd_kernel<\d, [01], (true|false)>", 256, 1),  # two-party split-digit kernel: four waves, one per SIMD
    (r"mk_latd_run_kernel<\d, [01]>", 256, 1),            # its later steps in one launch
    (r"mk_lat_run_kernel<\d, [01]>", 256, 1),             # the small-batch kernel's later steps in one launch
    (r"mk_quad_kernel<\d, [01], (true|false)>", 512, 1),  # one gate per workgroup (B <= CUs): one wave per
    (r"mk_quad_run_kernel<\d, [01]>", 512, 1),            # SIMD, so AGPRs may extend the register file
    (r"mk_quad2_kernel<[234], [01], false>", 256, 2),  # two workgroups per CU (B <= 4 x CUs, dg <= 4)
    (r"mk_quad2_run_kernel<[234], [01]>", 256, 2),
    (r"mk_quadp_run_kernel<\d, [01]>", 512, 1),          # party-parallel: a workgroup per party and CU
    (r"mk_quadp2_run_kernel<[234], [01]>", 256, 2),       # party-parallel, two workgroups per CU
    (r"mk_step_kernel<4, 0, false, true>", 256, 2),      # config-4 step (dg = 4, d_i scratch; spill-free since
                                                          # the alternating reload order)
    (r"mk_step_kernel<4, 1, false, false>", 256, 2),     # MK-LWE at dg = 4 (STD128_MKNTRU_LWE_4): keeps the asm
                                                          # forward products (MKACC_BFLY_C=2 is MK-NTRU only)
    (r"widereg2::step_kernel<[01], false>", 256, 2),     # config-5 FP64 step, two waves per gate
    (r"wide::step_kernel<[01], (true|false)>", 128, 4),    # 64-bit integer step (2^50 <= Q < 2^61)
    (r"extract_kernel|ks_mntru_kernel|ks_mklwe_kernel|mntru_head_kernel|mklwe_head_kernel", 256, 2),
]


@pytest.mark.parametrize("pattern,max_vgpr,min_occ", BUDGET)
def test_default_path_kernels_do_not_spill(pattern, max_vgpr, min_occ):
    hits = [r for r in _rows() if re.search(pattern, r["name"])]
    assert hits, f"no kernel matches {pattern!r} in the report"
    bad = []
    for r in hits:
        if r.get("VGPRs Spill", 0) or r.get("ScratchSize [bytes/lane]", 0):
            bad.append(f"{r['unit']}: {r['name']} spills (VGPR {r.get('VGPRs Spill')}, "
                       f"scratch {r.get('ScratchSize [bytes/lane]')} B/lane)")
        if r.get("VGPRs", 0) > max_vgpr or r.get("Occupancy [waves/SIMD]", 99) < min_occ:
            bad.append(f"{r['unit']}: {r['name']} at {r.get('VGPRs')} VGPRs / occupancy "
                       f"{r.get('Occupancy [waves/SIMD]')} (budget {max_vgpr} / {min_occ})")
    assert not bad, "\n".join(bad)


def test_headline_kernel_is_in_its_unit():
    """The headline kernel comes from the step2_dg3 unit, which is the one the
    scheduler flag applies to."""
    names = {(r["unit"], r["name"]) for r in _rows()}
    assert any(u == "step2_dg3" and "mk_step2_kernel<3, 0, false>" in n for u, n in names), sorted(names)[:20]


def test_step2_dg3_unit_uses_the_max_memory_clause_scheduler():
    from mkfhe_amd import build
    units = {name: defs for name, _, defs in build.UNITS}
    assert "-amdgpu-sched-strategy=max-memory-clause" in units["step2_dg3"]
    i = units["step2_dg3"].index("-amdgpu-sched-strategy=max-memory-clause")
    assert units["step2_dg3"][i - 1] == "-mllvm"


def test_guard_flags_a_spilling_report():
    """The parser and the budget catch a spill (the default scheduler's 6 spilled
    VGPRs at dg = 3, profiles/r3/ab_sched.txt, as the report would show it)."""
    fake = ("### unit step2_dg3\n"
            "x.hpp:1:1: remark: Function Name: _ZN12_GLOBAL__N_115mk_step2_kernelILi3ELi0ELb0EEEvNS_8StepArgsE "
            "[-Rpass-analysis=kernel-resource-usage]\n"
            "x.hpp:1:1: remark:     VGPRs: 256 [-Rpass-analysis=kernel-resource-usage]\n"
            "x.hpp:1:1: remark:     ScratchSize [bytes/lane]: 28 [-Rpass-analysis=kernel-resource-usage]\n"
            "x.hpp:1:1: remark:     Occupancy [waves/SIMD]: 2 [-Rpass-analysis=kernel-resource-usage]\n"
            "x.hpp:1:1: remark:     VGPRs Spill: 6 [-Rpass-analysis=kernel-resource-usage]\n")
    rows = parse_report(fake)
    assert len(rows) == 1 and rows[0]["VGPRs Spill"] == 6
    assert re.search(BUDGET[0][0], rows[0]["name"]), rows[0]["name"]
