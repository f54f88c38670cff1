"""CPU check of the two-waves-per-gate kernels' index maps
(mkfhe_amd/csrc/mkacc_layout2.hpp, used by widereg2::step_kernel): tools/widereg2_model.py runs the layouts, LDS word map (bank
groups of every LDS instruction the transposes use), per-lane twiddle indexing
and monomial split in exact integers against the oracle's NTT; the header's
constants must be the model's."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_widereg2_model_matches_oracle():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "widereg2_model.py")], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    for line in ("layouts ok", "forward transform ok", "inverse transform ok", "mono ok", "buffer schedule ok"):
        assert line in r.stdout


def test_layout_header_uses_the_model_word_map():
    src = open(os.path.join(ROOT, "mkfhe_amd", "csrc", "mkacc_layout2.hpp")).read()
    w = [int(x) for x in re.search(r"kW\[11\] = \{([^}]*)\}", src).group(1).split(",")]
    model = open(os.path.join(ROOT, "tools", "widereg2_model.py")).read()

    extra = dict((int(k), int(v)) for k, v in re.findall(r"bit\(p,(\d+)\)\*(\d+)", re.search(r"def pad\(p\):.*", model).group(0)))
    assert w == [(1 << k) + extra.get(k, 0) for k in range(11)]
    assert re.search(r"kBufE = (\d+)", src).group(1) == str(sum(w) + 1)
