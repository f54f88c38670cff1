#!/usr/bin/env python3
"""Throughput bench of the MI355X multi-key accumulator (EvalAcc = blind rotation).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--paramset NAME] [--batch B]

A "step" is one EvalAcc pass (all k*n accumulator steps) over one batch of B
independent synthetic gates per GPU, inputs resident in HBM.  N > 1 runs one
process per GPU (torch.distributed.run); rank 0 draws the bootstrapping keys
and broadcasts them once over RCCL; gates are sharded by rank with no
collective on the data path ("weak" scaling: B gates per GPU).

Rank 0 prints one JSON line (contract in the task statement); see DESIGN.md s6
for the roofline accounting.
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

# measured on this pool (tools/ubench_intops.hip, profiles/round1_ubench_intops.txt)
PEAK_SHOUP_MULMOD_TPS = 7.744e12     # 27-bit Shoup mod-mul / s, whole chip
PEAK_HBM_GBS = 8000.0                # MI355X_MICROARCH.md (spec)


def algorithmic_counts(k: int, n: int, dg: int, N: int = 2048, B: int = 1):
    """Per-launch algorithmic work of one accumulator step over B gates.

    mod-muls: (k+1)(dg+1) NTTs x N/2 log2 N butterflies (no N^-1 scaling: it is
    folded into the keys), k*N for acc*(X^c - 1), 2*dg*N key combination
    (d_i, f_i), (2k+1)*dg*N MAC products.  Bytes: the step's key block and P
    (read once per launch) + acc in/out per gate.
    """
    logn = N.bit_length() - 1
    ntt = (k + 1) * (dg + 1) * (N // 2) * logn
    mulmods = B * (ntt + k * N + 2 * dg * N + (2 * k + 1) * dg * N)
    key_bytes = 2 * dg * 2 * N * 4 + k * dg * N * 4
    bytes_ = key_bytes + B * (2 * k * N * 4 + 4)
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
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--n-override", type=int, default=0,
                    help="profiling aid: shorten the LWE dimension (fewer accumulator steps); not a bench config")
    return ap.parse_args()


def cpu_baseline(p, threads: int):
    """Oracle restatement (oracle/, 'port') timed on the host cores: `threads`
    independent gates, one per thread (bounded sample)."""
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
    orc.evalacc_batch(evk, pkey, ct, acc, threads)
    dt = time.perf_counter() - t0
    return {"value": threads / dt, "unit": "bootstraps/s", "cores": threads, "kind": "port",
            "sample": f"{threads} gates of {p.n}x{p.k}-step EvalAcc ({threads} threads, 1 gate each), "
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

    import mkfhe_amd as mk
    from mkfhe_amd import shard

    p = mk.paramset(args.paramset)
    if args.n_override:
        p.n = args.n_override
    eng = mk.MKAccumulatorEngine(p, device=local)
    B = args.batch

    # ---- keys: drawn on rank 0, broadcast once over RCCL (xGMI) ----
    evk_n = int(np.prod(eng.evk_shape))
    pkey_n = int(np.prod(eng.pkey_shape))
    keys = shard.broadcast_keys(evk_n + pkey_n, p.Q, seed=12345, device=f"cuda:{local}")
    keys_h = keys.cpu().numpy().view(np.uint32)
    eng.upload_keys(keys_h[:evk_n], keys_h[evk_n:])
    del keys, keys_h

    # ---- this rank's shard of synthetic gates, resident in HBM ----
    ct_h, acc_h = shard.synthetic_gates(eng, B, seed=1000 + rank)
    d_ct = torch.from_numpy(ct_h.view(np.int32)).to(f"cuda:{local}")
    d_in = torch.from_numpy(acc_h.view(np.int32)).to(f"cuda:{local}")
    d_out = torch.empty_like(d_in)
    stream = torch.cuda.ExternalStream(eng.stream_handle())

    for _ in range(args.warmup):
        eng.eval_batch_device(d_ct, d_in, d_out, B)
    eng.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        eng.eval_batch_device(d_ct, d_in, d_out, B)
    ev1.record(stream)
    eng.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    gpu_s = ev0.elapsed_time(ev1) / 1e3
    elapsed = torch.tensor([wall], dtype=torch.float64, device=f"cuda:{local}")
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    T = float(elapsed.item())

    # output sanity: residues stay canonical
    assert int(d_out.max().item()) < p.Q and int(d_out.min().item()) >= 0

    kn = p.k * p.n
    dg = p.digitsG - 1
    mm, by = algorithmic_counts(p.k, p.n, dg, p.N, B)
    per_launch_s = gpu_s / (args.steps * kn)   # the step kernel dominates (>99% of GPU time)
    result = {
        "metric": "MK NAND bootstraps/sec (EvalAcc blind rotation) at k=2,4,8 parties; 1/2/4/8 MI355X; bit-exact vs CPU",
        "value": world * B * args.steps / T,
        "unit": "bootstraps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * T / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32 (27-bit residues mod Q)",
        "data": "synthetic: uniform keys/ciphertexts, MNTRU test-vector accumulators",
        "config": {"workload": f"EvalAcc of {args.paramset} {p.k}-party {'MK-NTRU' if p.method == 0 else 'MK-LWE'} gate bootstraps "
                               f"(k={p.k}, n={p.n}, N={p.N}, dg={dg}); gate tail (extraction/ModSwitch/"
                               f"KeySwitch) not included",
                   "paramset": args.paramset, "batch_per_gpu": B, "global_batch": world * B,
                   "parallelism": f"gate-sharded x{world}"},
        "roofline": {"bound": "hbm", "achieved": by / per_launch_s / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": by / per_launch_s / 1e9 / PEAK_HBM_GBS,
                     "traffic": measured_traffic(args.paramset) if not args.n_override else None,
                     "kernel": "mk_step_kernel", "per_launch_us": per_launch_s * 1e6,
                     "bytes_per_launch": by},
        "roofline_valu": {"bound": "valu-int", "achieved": mm / per_launch_s / 1e12, "peak": PEAK_SHOUP_MULMOD_TPS / 1e12,
                          "unit": "T mod-mul/s", "frac": mm / per_launch_s / PEAK_SHOUP_MULMOD_TPS,
                          "mulmods_per_launch": mm},
    }
    if rank == 0 and world == 1 and args.cpu_baseline:
        thr = args.cpu_threads or min(16, os.cpu_count() or 1)
        result["cpu_baseline"] = cpu_baseline(p, thr)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
