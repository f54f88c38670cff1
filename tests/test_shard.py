"""Multi-rank plumbing on CPU (gloo, world size 2): gate sharding and the
one-time key broadcast that bench.py uses over RCCL on GPUs."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mkfhe_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("total,world", [(4096, 2), (4097, 2), (65536, 8), (5, 8), (0, 3), (1, 1)])
def test_shard_range_partitions(total, world):
    covered = []
    sizes = []
    for r in range(world):
        a, b = shard.shard_range(total, r, world)
        covered.extend(range(a, b))
        sizes.append(b - a)
    assert covered == list(range(total))
    assert max(sizes) - min(sizes) <= 1


def test_shard_range_rejects_bad_rank():
    with pytest.raises(ValueError):
        shard.shard_range(10, 2, 2)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        keys = shard.broadcast_keys(10000, 134176769, seed=7, device="cpu")
        h = keys.numpy().view(np.uint32)
        a, b = shard.shard_range(4096, rank, world)
        # max-over-ranks timing reduction as in bench.py
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        q.put((rank, int(h.astype(np.uint64).sum()), int(h.max()), a, b, float(t.item())))
    finally:
        dist.destroy_process_group()


def test_key_broadcast_and_sharding_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = shard.uniform_residues(10000, 134176769, 7)
    for rank, s, mx, a, b, t in res:
        assert s == int(expect.astype(np.uint64).sum())      # every rank holds rank 0's keys
        assert mx < 134176769
        assert t == float(world)                             # MAX over ranks
    assert [(a, b) for _, _, _, a, b, _ in res] == [(0, 2048), (2048, 4096)]
