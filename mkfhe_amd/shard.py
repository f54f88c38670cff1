"""Multi-GPU plumbing: gate sharding and the one-time key broadcast.

Gates are independent, so a batch shards by contiguous gate
ranges with no collective on the data path.  The only collective is the
one-time broadcast of the bootstrapping keys from rank 0 (RCCL over xGMI on
GPUs, gloo in the CPU tests).  Party-sharding is not used: HbProd mixes all k
accumulator polynomials every step.
"""
from __future__ import annotations

import numpy as np


def shard_range(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [start, stop) gate range of `rank`; sizes differ by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    q, r = divmod(total, world)
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


def word_dtype(Q: int):
    """Storage word of residues mod Q: uint32 up to 2^32, else uint64 (NATIVE_SIZE=64)."""
    return np.uint32 if Q <= (1 << 32) else np.uint64


def uniform_residues(nwords: int, Q: int, seed: int) -> np.ndarray:
    """Synthetic key material: uniform residues mod Q (uint32, or uint64 for Q > 2^32)."""
    return np.random.Generator(np.random.PCG64(seed)).integers(0, Q, size=nwords, dtype=word_dtype(Q))


def broadcast_keys(nwords: int, Q: int, seed: int, device: str = "cpu"):
    """Rank 0 draws `nwords` key words and broadcasts them once to every rank.

    Returns a torch int32 (int64 for Q > 2^32) tensor holding the bit pattern
    of the words on `device`.  Single-process runs skip the collective.
    """
    import torch
    import torch.distributed as dist

    multi = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    rank = dist.get_rank() if multi else 0
    wide = word_dtype(Q) == np.uint64
    if rank == 0:
        w = uniform_residues(nwords, Q, seed)
        t = torch.from_numpy(w.view(np.int64 if wide else np.int32)).to(device)
    else:
        t = torch.empty(nwords, dtype=torch.int64 if wide else torch.int32, device=device)
    if multi:
        dist.broadcast(t, src=0)
    return t


def mntru_test_vector(eng) -> np.ndarray:
    """BootstrapGateCore MNTRU accumulator init (binfhe-base-scheme.cpp:1093-1115):
    acc[0] = NTT(Rx) with Rx[j] = Q - (Q/8 + 1) for j < N/2 else Q/8 + 1; acc[u>0] = 0."""
    Q, N = eng.Q, eng.N
    q2p = Q // 8 + 1
    dt = word_dtype(Q)
    rx = np.where(np.arange(N) < N // 2, Q - q2p, q2p).astype(dt)
    acc = np.zeros((eng.k, N), dtype=dt)
    acc[0] = eng.ntt_forward(rx[None])[0]
    return acc


def synthetic_gates(eng, B: int, seed: int):
    """B synthetic gate inputs for `eng`: ct uniform (mod q for MKNTRU, mod 2N
    for the LWE/B variant) and the MNTRU test-vector accumulator."""
    rng = np.random.Generator(np.random.PCG64(seed))
    bound = eng.q if eng.method == 0 else 2 * eng.N
    ct = rng.integers(0, bound, size=(B, eng.k, eng.n), dtype=np.uint32)
    acc = np.broadcast_to(mntru_test_vector(eng), (B, eng.k, eng.N)).copy()
    return ct, acc
