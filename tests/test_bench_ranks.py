"""bench.py's multi-rank logic on CPU (gloo, world size 2): `bench.py --gpus 2`
launches its own ranks, broadcasts the keys, times a barrier-bracketed region,
reduces the time with MAX and sums the per-rank oracle checks -- with the GPU
engine and the oracle replaced by tests/bench_stub.py."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def _bench(*extra, env_extra=None):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    env.setdefault("OMP_NUM_THREADS", "1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--stub-engine", "--batch", "64",
           "--steps", "3", "--warmup", "1", *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, (json.loads(lines[-1]) if lines else None)


@pytest.mark.parametrize("stage,paramset", [("evalacc", "STD128_MKNTRU"), ("gate", "STD128_MKNTRU"),
                                            ("gate", "STD100_MKNTRU_LWE")])
def test_bench_spawns_two_ranks_and_checks_each_shard(stage, paramset):
    r, res = _bench("--stage", stage, "--paramset", paramset)
    assert r.returncode == 0, r.stderr[-3000:]
    assert res["n_gpus"] == 2 and res["steps"] == 3 and res["scaling"] == "weak"
    assert res["config"]["global_batch"] == 128
    # value = all ranks' gates / max-over-ranks time
    assert res["value"] == pytest.approx(2 * 64 * 3 / (res["ms_per_step"] * 3 / 1e3), rel=1e-9)
    assert res["parity_checked"] == 4 and res["parity_mismatches"] == 0   # 2 gates on each rank
    assert "cpu_baseline" not in res                                       # rank 0 at N = 1 only


def test_bench_fails_on_a_wrong_gate_of_rank_1():
    r, res = _bench("--stage", "evalacc", env_extra={"MKFHE_STUB_CORRUPT": "1"})
    assert r.returncode != 0
    assert res is not None and res["parity_checked"] == 4 and res["parity_mismatches"] == 1
    assert "parity FAILED" in r.stderr


def test_bench_n1_cpu_baseline_sample_grows_to_cpu_seconds():
    """N = 1: the cpu_baseline sample (and parity check) is extended with more gates of the
    timed batch until the oracle did --cpu-seconds of CPU work (the stub is instant, so the
    whole 64-gate batch is taken)."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--stub-engine", "--batch", "64",
           "--steps", "2", "--warmup", "1", "--n-override", "4", "--cpu-threads", "4"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["parity_checked"] == 64 and res["parity_mismatches"] == 0
    assert res["cpu_baseline"]["cores"] == 4 and "64 NAND gates" in res["cpu_baseline"]["sample"]
    r2 = subprocess.run(cmd + ["--cpu-seconds", "0"], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    res2 = json.loads([ln for ln in r2.stdout.splitlines() if ln.startswith("{")][-1])
    assert res2["parity_checked"] < 64   # one gate per usable core, not extended


# ---- world size 8: the driver's one-node scaling run, rehearsed on CPU (gloo) --------------

def _bench8(*extra):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.setdefault("OMP_NUM_THREADS", "1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--stub-engine", "--stub-shapes", "real",
           "--steps", "2", "--warmup", "1", "--stage", "gate", *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, (json.loads(lines[-1]) if lines else None)


def _usable_cores():
    sys.path.insert(0, ROOT)
    import bench
    return bench.cpu_info()["usable"]


def _check_ranks(res, world, B, want_bcast):
    assert res["n_gpus"] == world and res["config"]["global_batch"] == world * B
    ranks = res["ranks"]
    assert [r["rank"] for r in ranks] == list(range(world))
    # contiguous shards of B gates covering the global batch
    assert [tuple(r["gates"]) for r in ranks] == [(i * B, (i + 1) * B) for i in range(world)]
    # every rank received the same key material: rank 0's one broadcast
    assert all(r["keys_received_bytes"] == want_bcast for r in ranks) and res["keys_broadcast_bytes"] == want_bcast
    # 2 oracle-checked gates per rank, on (usable host cores // world) threads (at least 1)
    threads = max(1, min(2, _usable_cores() // world))
    assert all(r["oracle_threads"] == threads and r["checked"] == 2 and r["mismatches"] == 0 for r in ranks)
    assert res["parity_checked"] == 2 * world and res["parity_mismatches"] == 0
    assert res["value"] == pytest.approx(world * B * 2 / (res["ms_per_step"] * 2 / 1e3), rel=1e-9)


def test_bench_world8_headline_shapes():
    """The headline (STD128_MKNTRU, whole NAND gates) at world size 8 with the real key
    shapes: evk 150.6 MB + P + the 50 MB key-switching key broadcast once from rank 0."""
    import bench
    r, res = _bench8("--paramset", "STD128_MKNTRU", "--batch", "32")
    assert r.returncode == 0, r.stderr[-3000:]
    want = bench.key_broadcast_bytes(2, 765, 2048, 3, 2, 4, "gate", False, 45181)
    assert 200e6 < want < 202e6
    _check_ranks(res, 8, 32, want)


def test_bench_world8_config4_shard():
    """Config 4: 65,536 eight-party gates over 8 ranks, 8,192 per rank (BASELINE.json
    configs[3]); the LWE dimension is shortened for the CPU run (--n-override), the key
    broadcast is checked against the same formula, and at full size that formula gives
    the 803 MB bootstrapping key plus the 200 MB key-switching key."""
    import bench
    r, res = _bench8("--paramset", "STD128_MKNTRU_3", "--batch", "8192", "--n-override", "4")
    assert r.returncode == 0, r.stderr[-3000:]
    _check_ranks(res, 8, 8192, bench.key_broadcast_bytes(8, 4, 2048, 4, 2, 4, "gate", False, 45181))
    assert res["config"]["global_batch"] == 65536
    full_evk = bench.key_broadcast_bytes(8, 765, 2048, 4, 2, 4, "evalacc", False, 45181)
    full_gate = bench.key_broadcast_bytes(8, 765, 2048, 4, 2, 4, "gate", False, 45181)
    assert 802e6 < full_evk < 804e6                     # 802.7 MB (+ P)
    assert 200e6 < full_gate - full_evk < 201e6          # KSK [8][2048 x 4][765] u32
