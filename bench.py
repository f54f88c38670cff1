#!/usr/bin/env python3
"""Throughput bench of MK NAND gate bootstrapping on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--paramset NAME] [--batch B]
                    [--stage gate|evalacc]

A "step" is one pass over a batch of B independent synthetic NAND gates per
GPU with inputs resident in HBM.  --stage gate (default) runs the whole
EvalBinGate of the reference -- gate head, BootstrapGateCore (test vector +
EvalAcc, the blind rotation) and the tail (extraction, ModSwitch, KeySwitch2 /
KeySwitch); --stage evalacc runs the accumulator alone.  N > 1 runs one process
per GPU (torch.distributed.run): rank 0 draws the bootstrapping and
key-switching keys and broadcasts them once over RCCL; gates are sharded by
rank with no collective on the data path ("weak" scaling: B gates per GPU).

Rank 0 prints one JSON line (contract in the task statement); DESIGN.md s4.4
and s5 give the roofline accounting.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]

# measured on this pool (tools/ubench_intops.hip, profiles/round1_ubench_intops.txt)
PEAK_SHOUP_MULMOD_TPS = 7.744e12     # 27-bit Shoup mod-mul / s, whole chip
PEAK_HBM_GBS = 8000.0                # MI355X_MICROARCH.md (spec)
Q50 = 1125899906826241               # config 5 stress modulus


def algorithmic_counts(k: int, n: int, dg: int, nk: int, N: int = 2048, B: int = 1, word: int = 4):
    """Per-launch algorithmic work of one accumulator step over B gates.

    mod-muls: (k+1)(dg+1) NTTs x N/2 log2 N butterflies (no N^-1 scaling: it is
    folded into the keys), k*N for acc*(X^c - 1), 2*dg*N key combination
    (d_i, f_i; XZW only), (2k+1)*dg*N MAC products.  Bytes: the step's key
    block (nk key sets of [dg][2][N]) and P, read once per launch, plus the
    accumulator in/out and the exponent per gate.
    """
    logn = N.bit_length() - 1
    ntt = (k + 1) * (dg + 1) * (N // 2) * logn
    comb = 2 * dg * N if nk == 2 else 0
    mulmods = B * (ntt + k * N + comb + (2 * k + 1) * dg * N)
    key_bytes = (nk * dg * 2 * N + k * dg * N) * word
    bytes_ = key_bytes + B * (2 * k * N * word + 4)
    return mulmods, bytes_


def measured_traffic(paramset: str):
    """Per-launch HBM bytes of the step kernel from the committed PMC record
    (profiles/traffic_<paramset>.json, written by tools/pmc_summary.py from
    separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes), or None."""
    f = os.path.join(ROOT, "profiles", f"traffic_{paramset}.json")
    if not os.path.exists(f):
        return None
    return json.load(open(f))["traffic_bytes"]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--paramset", default="STD128_MKNTRU")
    ap.add_argument("--batch", type=int, default=4096, help="gates per GPU")
    ap.add_argument("--stage", choices=["gate", "evalacc"], default="gate")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--q-bits", type=int, default=0, choices=[0, 50],
                    help="50: config 5 stress -- the paramset's shape with the 50-bit Q = 1125899906826241 and "
                         "B_g = 2^10 in 64-bit words (EvalAcc on the 64-bit word path)")
    ap.add_argument("--n-override", type=int, default=0,
                    help="profiling aid: shorten the LWE dimension (fewer accumulator steps); not a bench config")
    return ap.parse_args()


def cpu_baseline(p, threads: int, stage: str, ks):
    """The oracle restatement (oracle/, 'port') timed on the host cores:
    `threads` independent gates, one per thread (bounded sample).  For the gate
    stage the tail is the same contraction the oracle pins (tests/test_gate.py),
    done in numpy; it is <2% of the gate."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    pyoracle.build()
    method = pyoracle.XZW if p.method == 0 else pyoracle.XZW_B
    orc = pyoracle.Oracle(method, p.k, p.n, p.N, p.Q, p.q, p.baseG, p.digitsG, p.root)
    evk = pyoracle.fill_uniform(int(np.prod(orc.evk_shape)), p.Q, 101)
    pkey = pyoracle.fill_uniform(int(np.prod(orc.pkey_shape)), p.Q, 102)
    bound = p.q if p.method == 0 else 2 * p.N
    ct = pyoracle.fill_uniform(threads * p.k * p.n, bound, 103).reshape(threads, p.k, p.n)
    acc = np.broadcast_to(orc.mntru_testvector(4), (threads, p.k, p.N)).copy()
    t0 = time.perf_counter()
    out = orc.evalacc_batch(evk, pkey, ct, acc, threads)
    if stage == "gate":
        qKS, baseKS, dks = ks
        ksk = pyoracle.fill_uniform(p.k * p.N * dks * p.n, qKS, 104).reshape(p.k, p.N * dks, p.n).astype(np.int64)
        for g in range(threads):
            ext = orc.extract(out[g])
            ms = np.vectorize(lambda v: pyoracle.round_qQ(int(v), qKS, p.Q), otypes=[np.int64])(ext)
            digits = np.stack([(ms // baseKS ** t) % baseKS for t in range(dks)], axis=-1).reshape(p.k, -1)
            _ = np.stack([(digits[u] @ ksk[u]) % qKS for u in range(p.k)])
    dt = time.perf_counter() - t0
    what = "NAND gates (EvalAcc + extraction/ModSwitch/KeySwitch)" if stage == "gate" else "EvalAcc"
    return {"value": threads / dt, "unit": "bootstraps/s", "cores": threads, "kind": "port",
            "sample": f"{threads} {what} of {p.n}x{p.k} accumulator steps, one per thread on {threads} threads, "
                      f"{dt:.2f} s wall, CPU {os.uname().machine} nproc={os.cpu_count()}"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world)
    dev = f"cuda:{local}"

    import mkfhe_amd as mk
    from mkfhe_amd import shard

    p = mk.paramset(args.paramset)
    if args.n_override:
        p.n = args.n_override
    if args.q_bits == 50:   # SURVEY.md s8 config 5 stress (s6: reference CPU 0.568 s / EvalAcc at k=2, n=560)
        p.Q, p.baseG, p.digitsG, p.root = Q50, 1 << 10, 0, 0
        args.stage = "evalacc"   # the 64-bit word path covers the accumulator
    eng = mk.MKAccumulatorEngine(p, device=local)
    p = eng.params
    wide = eng.wide
    word = 8 if p.Q > (1 << 32) else 4
    B = args.batch
    lwe = p.method != mk.MKNTRU
    qKS, baseKS = p.q, 32                     # modKS = mod and baseKS = 32 in every MK set (binfhecontext.cpp:129-144)
    dks = int(np.ceil(np.log(qKS) / np.log(baseKS)))

    # ---- keys: drawn on rank 0, broadcast once over RCCL (xGMI) ----
    evk_n = int(np.prod(eng.evk_shape))
    pkey_n = int(np.prod(eng.pkey_shape))
    keys = shard.broadcast_keys(evk_n + pkey_n, p.Q, seed=12345, device=dev)
    keys_h = keys.cpu().numpy().view(np.uint64 if word == 8 else np.uint32)
    eng.upload_keys(keys_h[:evk_n], keys_h[evk_n:])
    del keys, keys_h
    if args.stage == "gate":
        if lwe:
            na = p.k * p.N * baseKS * dks * p.n
            nb = p.k * p.N * baseKS * dks
            ksk = shard.broadcast_keys(na + nb, qKS, seed=23456, device=dev).cpu().numpy().view(np.uint32)
            eng.upload_ksk_mklwe(ksk[:na], ksk[na:], qKS, baseKS, p.n)
        else:
            nk = p.k * p.N * dks * p.n
            ksk = shard.broadcast_keys(nk, qKS, seed=23456, device=dev).cpu().numpy().view(np.uint32)
            eng.upload_ksk_mntru(ksk, qKS, baseKS, p.n)
        del ksk

    # ---- this rank's shard of synthetic gates, resident in HBM ----
    rng = np.random.Generator(np.random.PCG64(1000 + rank))

    def dev_u32(a):
        if a.dtype == np.uint64:
            return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
        return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).to(dev)

    stream = torch.cuda.ExternalStream(eng.stream_handle())
    if args.stage == "gate":
        kn = p.k * p.n
        d_a1 = dev_u32(rng.integers(0, p.q, size=(B, kn)))
        d_a2 = dev_u32(rng.integers(0, p.q, size=(B, kn)))
        d_nand = dev_u32(rng.integers(0, p.q, size=kn))
        d_b1 = dev_u32(rng.integers(0, p.q, size=B)) if lwe else None
        d_b2 = dev_u32(rng.integers(0, p.q, size=B)) if lwe else None
        d_oa = torch.empty((B, p.k * p.n), dtype=torch.int32, device=dev)
        d_ob = torch.empty(B, dtype=torch.int32, device=dev) if lwe else None

        def run_step():
            eng.eval_nand_device(d_nand, d_a1, d_b1, d_a2, d_b2, d_oa, d_ob, B)
    else:
        ct_h, acc_h = shard.synthetic_gates(eng, B, seed=1000 + rank)
        d_ct, d_in = dev_u32(ct_h), dev_u32(acc_h)
        d_out = torch.empty_like(d_in)

        def run_step():
            eng.eval_batch_device(d_ct, d_in, d_out, B)

    for _ in range(args.warmup):
        run_step()
    eng.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run_step()
    eng.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    elapsed = torch.tensor([wall], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    T = float(elapsed.item())

    # output sanity: residues stay canonical
    if args.stage == "gate":
        assert int(d_oa.max().item()) < qKS and int(d_oa.min().item()) >= 0
    else:
        hi = d_out.view(torch.int64) if word == 8 else d_out
        assert int(hi.max().item()) < p.Q and int(hi.min().item()) >= 0

    # ---- dominant kernel (the accumulator step) timed live with HIP events on
    # the engine stream: one EvalAcc pass = k*n step launches (+2 tiny kernels)
    ct_h, acc_h = shard.synthetic_gates(eng, B, seed=2000 + rank)
    d_ct, d_in = dev_u32(ct_h), dev_u32(acc_h)
    d_out = torch.empty_like(d_in)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    eng.eval_batch_device(d_ct, d_in, d_out, B)
    ev1.record(stream)
    eng.sync()
    kn_steps = p.k * p.n
    per_launch_s = ev0.elapsed_time(ev1) / 1e3 / kn_steps

    dg = p.digitsG - 1
    nk = 1 if lwe else 2
    mm, by = algorithmic_counts(p.k, p.n, dg, nk, p.N, B, word)
    stage_txt = ("NAND gates: head + BootstrapGateCore (EvalAcc) + extraction/ModSwitch/"
                 f"{'KeySwitch' if lwe else 'KeySwitch2'}") if args.stage == "gate" else "EvalAcc (blind rotation) only"
    result = {
        "metric": METRIC,
        "value": world * B * args.steps / T,
        "unit": "bootstraps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * T / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64 (50-bit residues mod Q)" if word == 8 else "u32 (27-bit residues mod Q)",
        "data": "synthetic: uniform keys, key-switching keys and ciphertexts (seeded)",
        "config": {"workload": f"{args.paramset} {p.k}-party {'MK-LWE' if lwe else 'MK-NTRU'} {stage_txt} "
                               f"(k={p.k}, n={p.n}, N={p.N}, dg={dg}"
                               + (f", Q={p.Q} in 64-bit words, B_g=2^{p.baseG.bit_length() - 1})" if wide else ")"),
                   "paramset": args.paramset, "stage": args.stage, "batch_per_gpu": B, "global_batch": world * B,
                   "parallelism": f"gate-sharded x{world}"},
        "roofline": {"bound": "hbm", "achieved": by / per_launch_s / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": by / per_launch_s / 1e9 / PEAK_HBM_GBS,
                     "traffic": measured_traffic(args.paramset) if not (args.n_override or wide) else None,
                     "kernel": "wide::step_kernel" if wide else "mk_step_kernel",
                     "per_launch_us": per_launch_s * 1e6,
                     "bytes_per_launch": by},
        # the VALU peak is the measured 32-bit Shoup rate: not a bound for 64-bit words
        "roofline_valu": None if wide else {
            "bound": "valu-int", "achieved": mm / per_launch_s / 1e12, "peak": PEAK_SHOUP_MULMOD_TPS / 1e12,
            "unit": "T mod-mul/s", "frac": mm / per_launch_s / PEAK_SHOUP_MULMOD_TPS, "mulmods_per_launch": mm},
    }
    if rank == 0 and world == 1 and args.cpu_baseline:
        thr = args.cpu_threads or min(16, os.cpu_count() or 1)
        result["cpu_baseline"] = cpu_baseline(p, thr, args.stage, (qKS, baseKS, dks))
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
