"""CPU stand-ins for bench.py's engine and oracle checker (tests/test_bench_ranks.py).

`python bench.py --stub-engine` runs bench.py's real rank logic -- launcher,
key broadcast, per-rank shards, warmup, barrier-bracketed timing, max-over-ranks
reduction, the per-rank check of G gates spread over the batch and the sum over ranks --
over gloo on the CPU, with only the GPU engine and the oracle replaced by these
toy functions.  The toy "accumulator" depends on the broadcast keys and on every
input word, so a rank that received the wrong keys or a mis-sharded batch
fails the check.  MKFHE_STUB_CORRUPT=<rank> corrupts gate 0 of that rank.
"""
from __future__ import annotations

import os
import types

import numpy as np
import torch

Q, QLWE = 134176769, 45181


def _digest(evk, pkey) -> int:
    return int((np.asarray(evk, dtype=np.uint64).sum() + np.asarray(pkey, dtype=np.uint64).sum()) % Q)


class StubEngine:
    """--stub-shapes toy (default): k = 2, n = 8, N = 16; real: the parameter set's own
    k, n (or --n-override), N and digit count, so the key broadcast has its real size."""

    def __init__(self, args):
        lwe = "_LWE" in args.paramset
        if getattr(args, "stub_shapes", "toy") == "real":
            import mkfhe_amd as mk
            r = mk.paramset(args.paramset)
            self.params = types.SimpleNamespace(method=2 if lwe else 0, k=r.k, n=args.n_override or r.n, N=r.N,
                                                Q=Q, q=r.q, baseG=r.baseG, digitsG=r.digitsG, root=0)
        else:
            self.params = types.SimpleNamespace(method=2 if lwe else 0, k=2, n=8, N=16, Q=Q, q=QLWE, baseG=128,
                                                digitsG=4, root=0)
        p = self.params
        self.method, self.k, self.n, self.N, self.Q, self.q = p.method, p.k, p.n, p.N, p.Q, p.q
        self.wide = False
        self.nk = 1 if lwe else 2
        self.evk_shape = (p.k, self.nk, p.n + 1, p.digitsG - 1, 2, p.N)
        self.pkey_shape = (p.k, p.digitsG - 1, p.N)
        self.kd = None
        self.rank = int(os.environ.get("RANK", 0))

    def upload_keys_device(self, d_evk, d_pkey):
        assert d_evk.numel() == int(np.prod(self.evk_shape)) and d_pkey.numel() == int(np.prod(self.pkey_shape))
        self.kd = int((d_evk.to(torch.int64).sum() + d_pkey.to(torch.int64).sum()).item() % Q)

    def upload_ksk_device(self, qKS, baseKS, n_out, d_ksk=None, d_A=None, d_B=None):
        assert (d_ksk is not None) != (d_A is not None and d_B is not None)
        self.ks = (qKS, baseKS, n_out)

    def ntt_forward(self, a):
        return np.array(a, copy=True)

    def _corrupt(self, t):
        if os.environ.get("MKFHE_STUB_CORRUPT") == str(self.rank):
            t.view(-1)[0] += 1

    def eval_batch_device(self, d_ct, d_in, d_out, B):
        s = d_ct.to(torch.int64).reshape(B, -1).sum(dim=1).reshape(B, 1, 1)
        d_out.copy_(((d_in.to(torch.int64) + s + self.kd) % Q).to(d_out.dtype))
        self._corrupt(d_out)

    def eval_nand_device(self, d_nand, d_a1, d_b1, d_a2, d_b2, d_out_a, d_out_b, B):
        a = d_a1.to(torch.int64) + d_a2.to(torch.int64) + d_nand.to(torch.int64).unsqueeze(0) + self.kd
        d_out_a.copy_((a % QLWE).to(d_out_a.dtype))
        if d_out_b is not None:
            d_out_b.copy_(((d_b1.to(torch.int64) + d_b2.to(torch.int64) + self.kd) % QLWE).to(d_out_b.dtype))
        self._corrupt(d_out_a)

    def sync(self):
        pass

    def stream_handle(self):
        return 0


class StubChecker:
    kind = "stub"

    def __init__(self, p, lwe):
        self.p, self.lwe = p, lwe

    def evalacc(self, evk, pkey, ct, acc, threads):
        kd = _digest(evk, pkey)
        s = ct.reshape(ct.shape[0], -1).sum(axis=1).reshape(-1, 1, 1)
        return (acc + s + kd) % Q

    def gates(self, keys, ksk, inputs, threads, ks):
        kd = _digest(*keys)
        a = (inputs["a1"].astype(np.uint64) + inputs["a2"] + inputs["nand"][None] + kd) % QLWE
        b = (inputs["b1"].astype(np.uint64) + inputs["b2"] + kd) % QLWE if self.lwe else None
        return a, b
