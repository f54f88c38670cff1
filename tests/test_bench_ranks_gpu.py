"""bench.py's N > 1 path on MI355X hardware: two ranks sharing the box's one GPU
(`--shared-gpu`: every rank runs the real engine on device 0, the collectives go
over gloo because RCCL refuses two ranks on one device).  Rank 0 draws and
broadcasts the key material into device tensors, each rank builds its own
engine, uploads the keys from those tensors, runs its contiguous shard, and the
oracle checks gates of every rank's shard -- the plumbing the driver's 8-GPU run
uses, on real kernels.  (Not a scaling measurement: both ranks share one GPU.)"""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


@pytest.mark.gpu
def test_bench_two_ranks_on_one_gpu():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    B = 64
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--shared-gpu", "--batch", str(B),
           "--steps", "2", "--warmup", "1", "--n-override", "8", "--check-gates", "2"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["n_gpus"] == 2 and res["config"]["global_batch"] == 2 * B
    ranks = res["ranks"]
    assert [tuple(x["gates"]) for x in ranks] == [(0, B), (B, 2 * B)]
    assert all(x["keys_received_bytes"] == res["keys_broadcast_bytes"] > 0 for x in ranks)
    assert all(x["checked"] >= 1 and x["mismatches"] == 0 for x in ranks)
    assert res["parity_mismatches"] == 0 and res["parity_checked"] == sum(x["checked"] for x in ranks)
    assert "rehearsal" in res["config"]["parallelism"]
