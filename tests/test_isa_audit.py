"""Build-level guard (CPU, no GPU): the built engine library must have no
16-byte store whose data registers are rewritten within 2 wait states -- the
gfx950 VMEM store-data hazard that silently corrupted the second co-resident
workgroup's accumulators (tools/isa_audit.py) -- and no SALU
use of VCC within 8 wait states of an inline-asm multiply-add that writes its
carry-out to VCC (the intermittent small-batch kernel defect)."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

LIB = os.path.join(ROOT, "mkfhe_amd", "lib", "libmkfhe_amd.so")
TOOLS = ["/opt/rocm/lib/llvm/bin/llvm-objcopy", "/opt/rocm/lib/llvm/bin/clang-offload-bundler",
         "/opt/rocm/lib/llvm/bin/llvm-objdump"]


@pytest.mark.skipif(not os.path.exists(LIB) or not all(os.path.exists(t) for t in TOOLS),
                    reason="engine library or LLVM tools absent")
def test_no_store_data_hazards():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "isa_audit.py"), LIB],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert " 0 data-register hazards" in r.stdout
    assert " 0 VCC carry-out hazards" in r.stdout


def test_audit_flags_a_hazard():
    """The checker itself: a dwordx4 store followed by a write of its data register."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_audit
    bad = """0000000000001000 <k>:
	buffer_store_dwordx4 v[0:3], v194, s[0:3], s93 offen
	v_mul_lo_u32 v2, s37, v8
"""
    ok = """0000000000001000 <k>:
	buffer_store_dwordx4 v[0:3], v194, s[0:3], s93 offen
	s_nop 1
	v_mul_lo_u32 v2, s37, v8
	global_store_dwordx4 v[10:11], v[4:7], off
	v_add_u32_e32 v8, v1, v2
"""
    assert len(isa_audit.audit(bad)[1]) == 1
    assert isa_audit.audit(ok) == (2, [], 0)


def test_audit_flags_a_vcc_carry_hazard():
    """The checker itself: an SALU write of VCC (a branch condition) right after a
    multiply-add whose carry-out goes to VCC -- the mk_lat_kernel defect."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_audit
    bad = """0000000000001000 <k>:
	v_mad_u64_u32 v[2:3], vcc, v0, s78, v[128:129]
	s_andn2_b64 vcc, exec, s[0:1]
	s_cbranch_vccnz 12268
"""
    ok = """0000000000001000 <k>:
	v_mad_u64_u32 v[2:3], vcc, v0, s78, v[128:129]
	s_nop 7
	s_andn2_b64 vcc, exec, s[0:1]
	s_cbranch_vccnz 12268
"""
    assert isa_audit.audit(bad)[2] == 1
    assert isa_audit.audit(ok) == (0, [], 0)
