"""The reference's r-defect in KeyGenXZW (mk-acc-xzw.cpp:141-167): a DggR
sample r != 0 enters f as g_t * r but d only as the scalar r^[t] * CRS_t, so
the key breaks every gate that uses it.  Pinned on a key set
the 1000-set fresh-key run found (profiles/r3/fresh_key_rate_STD128_MKNTRU_1000.jsonl,
set 177): replaying its entropy master must regenerate the same defective key
and the same wrong gates through the CPU oracle -- this checks the entropy
journal's determinism and that the restatement keeps the reference's defect."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))

MASTER = "c5681f85f6e98f1ed21bdcb0d9ad223c8111d67f4e8567c3c4a5abc97eee0275"


def test_replayed_key_set_has_the_recorded_defect(oracle):
    import fresh_key_rate as F
    from mkfhe_amd import keys as K
    p = K.paramset("STD128_MKNTRU", 0)
    orc = oracle.Oracle(oracle.XZW, p.acc.k, p.acc.n, 2048, p.acc.Q, p.acc.q, p.acc.baseG)
    K.entropy_replay()
    saved = K.entropy_get()
    try:
        K.entropy_set(MASTER)
        dec, bk = F.example_run(K, oracle, p, orc, False, min(8, os.cpu_count() or 1))
        assert F.r_defects(oracle, p, bk) == [(1, 1, 122)]
        assert dec == [0, 3, 3, 3]       # recorded: all four NAND gates wrong
    finally:
        K.entropy_set(saved[0], saved[1])


def test_r_defect_scan_is_clean_on_a_normal_set(oracle):
    import fresh_key_rate as F
    from mkfhe_amd import keys as K
    p = K.paramset("STD100_MKNTRU", 0)
    K.entropy_replay()
    saved = K.entropy_get()
    try:
        K.entropy_set("00" * 32)
        sk = K.mntru_keygen(p, 0)
        bk = K.bt_keygen(p, sk, seed=0)
        assert F.r_defects(oracle, p, bk) == []
        assert bk.evk.shape[:3] == (p.acc.k, 2, p.acc.n + 1) and np.any(bk.evk)
    finally:
        K.entropy_set(saved[0], saved[1])


def test_keygen_reports_rejects_or_resamples_the_defective_key(oracle):
    """the r-defect is reported at the API.  On the recorded key set
    (set 177) the default policy keeps the reference's keys bit for bit and counts
    the one defective key; "reject" raises KeyDefectError; "resample" redraws r in
    that slot only, after which all four NAND gates decrypt correctly."""
    import fresh_key_rate as F
    from mkfhe_amd import keys as K
    p = K.paramset("STD128_MKNTRU", 0)
    orc = oracle.Oracle(oracle.XZW, p.acc.k, p.acc.n, 2048, p.acc.Q, p.acc.q, p.acc.baseG)
    K.entropy_replay()
    saved = K.entropy_get()
    try:
        K.entropy_set(MASTER)
        sk = K.mntru_keygen(p, 0)
        kept = K.bt_keygen(p, sk, seed=0)                 # the default: bit-faithful
        assert kept.rdefects == 1
        K.entropy_set(MASTER)
        sk = K.mntru_keygen(p, 0)
        with pytest.raises(K.KeyDefectError, match="nonzero DggR") as rejected:
            K.bt_keygen(p, sk, seed=0, rdefect="reject")
        assert rejected.value.rdefects == 1               # the count survives the rejection
        K.entropy_set(MASTER)
        dec, bk = F.example_run(K, oracle, p, orc, False, min(8, os.cpu_count() or 1), rdefect="resample")
        assert bk.rdefects == 1 and F.r_defects(oracle, p, bk) == []
        assert dec == [1, 1, 1, 0]                        # NAND of (0,0), (0,1), (1,0), (1,1)
        # only the defective slot (u = 1, s = 1, i = 122) differs from the reference's keys
        diff = np.argwhere(np.any(bk.evk != kept.evk, axis=(3, 4, 5)))
        assert diff.tolist() == [[1, 1, 122]]
    finally:
        K.entropy_set(saved[0], saved[1])
