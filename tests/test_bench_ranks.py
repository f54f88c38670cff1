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
