"""The party-parallel kernel's share ring (mkacc_quad.hpp, quadp_step) under random
schedules: every step finishes, no share of another step is ever accepted, and the
three ordering rules the kernel relies on are each necessary (tools/quadp_protocol.py)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import quadp_protocol as P  # noqa: E402


def test_ring_is_clean():
    assert P.check(seeds=10, ppws=(1, 2, 3)) == []
    assert P.check(seeds=6, ppws=(1, 2), preload=True) == []   # MKACC_QUADP_PRELOAD=1


def test_each_rule_is_needed():
    assert P.check(seeds=30, own_write=False)
    assert P.check(seeds=30, takeover_wait=False)
    assert P.check(seeds=30, reload=False, preload=True)
