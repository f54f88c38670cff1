#!/usr/bin/env python3
"""Throughput bench of MK NAND gate bootstrapping on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--paramset NAME] [--batch B]
                    [--stage gate|evalacc] [--q-bits 50]

A "step" is one pass over a batch of B independent synthetic NAND gates per
GPU with inputs resident in HBM.  --stage gate (default) runs the whole
EvalBinGate of the reference -- gate head, BootstrapGateCore (test vector +
EvalAcc, the blind rotation) and the tail (extraction, ModSwitch, KeySwitch2 /
KeySwitch); --stage evalacc runs the accumulator alone.

Multi-GPU: one process per GPU.  Under torch.distributed.run the ranks come
from the environment; `--gpus N` without WORLD_SIZE launches the N ranks
itself (a child torch.distributed.run, before anything touches a GPU).  Rank 0
draws the bootstrapping and key-switching keys and broadcasts them once over
RCCL; every rank uploads them straight from the received device buffer
(mkacc_upload_keys_device, mkacc_upload_ksk_*_device).  Gates are sharded by rank with no collective on
the data path ("weak" scaling: B gates per GPU).

Proof of the timed run: after timing, every rank copies back the outputs of
G gates spread over ITS timed batch and recomputes them with the CPU oracle
(oracle/, the checker) from the same inputs and keys; rank 0 reports
`parity_checked` / `parity_mismatches` summed over ranks and the run fails on a
mismatch.  At N = 1 those G gates, one per host core, are also the CPU
baseline (`cpu_baseline`, kind "port": this repo's restatement of the
reference path).

Rank 0 prints one JSON line (contract in the task statement); DESIGN.md s4.4
and s5 give the roofline accounting.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]

# measured on this pool (tools/ubench_intops.hip, profiles/round1_ubench_intops.txt)
PEAK_SHOUP_MULMOD_TPS = 7.744e12     # 27-bit Shoup mod-mul / s, whole chip
# 64-bit word path (tools/ubench_wide.hip, profiles/r2/ubench_wide.txt, 50-bit Q):
PEAK_FP64_MULMOD_TPS = 5.7455e12     # exact FP64 product (mkacc_fp64.hpp, widereg2 kernel) / s
PEAK_INT64_MULMOD_TPS = 1.7433e12    # limb-built 64-bit Shoup product (mkacc_wide.hpp) / s
PEAK_HBM_GBS = 8000.0                # MI355X_MICROARCH.md (spec)
Q50 = 1125899906826241               # config 5 stress modulus
REF_CPU_S_PER_EVALACC = {            # reference EvalAcc, 1 core of the survey container
    "STD100_MKNTRU": 0.274, "STD128_MKNTRU": 0.475, "STD100_MKNTRU_LWE": 0.215,
    "STD100_MKNTRU_LWE_2": 0.721, "STD128_MKNTRU_3": 6.750, "STD100_MKNTRU_3": 2.872}
# oracle / reference single-thread EvalAcc time, read from the calibration record
# (tools/oracle_calib.py -> profiles/oracle_calibration.json).  A
# CROSS-MACHINE estimate: the oracle was timed on this repo's Intel Xeon (AVX-512)
# container, the reference by the survey on an 8-vCPU AMD EPYC container; the reference
# cannot be rebuilt here to time both on one CPU.
CALIBRATION_RECORD = "profiles/oracle_calibration.json"


def oracle_over_ref() -> dict:
    rec = json.load(open(os.path.join(ROOT, CALIBRATION_RECORD)))
    return {k: v["oracle_over_reference"] for k, v in rec.items() if isinstance(v, dict) and "oracle_over_reference" in v}


def calibration() -> dict:
    rec = json.load(open(os.path.join(ROOT, CALIBRATION_RECORD)))
    return {"same_machine": rec.get("same_machine", False), "oracle_cpu": rec.get("oracle_cpu"),
            "reference_cpu": rec.get("reference_cpu"), "record": CALIBRATION_RECORD}


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


def key_broadcast_bytes(k: int, n: int, N: int, dg: int, nk: int, word: int, stage: str, lwe: bool, qKS: int,
                        baseKS: int = 32) -> int:
    """Bytes rank 0 broadcasts once (run_rank): the bootstrapping key evk [k][nk][n+1][dg][2][N]
    and P [k][dg][N] in `word`-byte words, and for whole gates the key-switching key as u32 --
    MK-NTRU KSK [k][N dks][n] (KSK2's multiples j KSK are formed by the kernel,
    mntru-pke.cpp:744-755), MK-LWE A [k][N][baseKS][dks][n] and B [k][N][baseKS][dks]."""
    dks = int(np.ceil(np.log(qKS) / np.log(baseKS)))
    b = (k * nk * (n + 1) * dg * 2 * N + k * dg * N) * word
    if stage == "gate":
        b += (k * N * baseKS * dks * (n + 1) if lwe else k * N * dks * n) * 4
    return b


def library_kernel_ids() -> dict:
    """{demangled kernel: isa id} of the engine library this process runs
    (mkfhe_amd/build.py writes it next to the library, tools/kernel_isa.py)."""
    from mkfhe_amd import _lib
    f = _lib.LIB_PATH[:-3] + ".kernel_isa.json"
    return json.load(open(f)) if os.path.exists(f) else {}


def measured_traffic(paramset: str, kernel: str, algorithmic: float) -> dict:
    """Per-launch HBM bytes of the step kernel from the committed PMC record
    (profiles/traffic_<paramset>.json, written by tools/pmc_summary.py from
    separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes).  `bytes` is None
    unless the record was taken of this very kernel: same name, and the same
    machine code (isa id) as the kernel in the library being benched."""
    f = os.path.join(ROOT, "profiles", f"traffic_{paramset}.json")
    if not os.path.exists(f):
        return {"bytes": None, "why": f"no record profiles/traffic_{paramset}.json"}
    rec = json.load(open(f))
    if rec.get("kernel") != kernel:
        return {"bytes": None, "why": f"record is of {rec.get('kernel')}, benched kernel is {kernel}"}
    sym, isa = rec.get("kernel_symbol"), rec.get("kernel_isa")
    have = library_kernel_ids().get(sym) if sym else None
    if not isa or have != isa:
        return {"bytes": None, "why": f"record's kernel isa id {isa} differs from the library's {have} ({sym})"}
    t = rec["traffic_bytes"]
    return {"bytes": t, "over_algorithmic": t / algorithmic, "kernel_symbol": sym, "kernel_isa": isa,
            "record": f"profiles/traffic_{paramset}.json", "pmc_source": rec.get("source")}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--paramset", default="STD128_MKNTRU")
    ap.add_argument("--batch", type=int, default=4096, help="gates per GPU")
    ap.add_argument("--stage", choices=["gate", "evalacc"], default="gate")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: every usable host core")
    ap.add_argument("--check-gates", type=int, default=0,
                    help="gates per rank recomputed by the oracle (0: one per host core at N=1, 2 per rank at N>1)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="N=1: oracle CPU work (threads x wall seconds) of the cpu_baseline sample; more gates of "
                         "the timed batch are recomputed (and parity-checked) until it is reached")
    ap.add_argument("--q-bits", type=int, default=0, choices=[0, 50],
                    help="50: config 5 stress -- the paramset's shape with the 50-bit Q = 1125899906826241 and "
                         "B_g = 2^10 in 64-bit words (EvalAcc on the 64-bit word path)")
    ap.add_argument("--n-override", type=int, default=0,
                    help="profiling aid: shorten the LWE dimension (fewer accumulator steps); not a bench config")
    ap.add_argument("--stub-engine", action="store_true",
                    help="test aid (tests/test_bench_ranks.py): CPU stand-in engine + gloo, to exercise the rank logic")
    ap.add_argument("--stub-shapes", choices=["toy", "real"], default="toy",
                    help="test aid: the stand-in engine's key and gate shapes (real: the parameter set's)")
    ap.add_argument("--shared-gpu", action="store_true",
                    help="rehearsal aid on a one-GPU box: every rank runs the real engine on device 0 and the "
                         "collectives go over gloo (RCCL refuses two ranks on one device); a plumbing check of "
                         "the N > 1 path on hardware, not a scaling measurement")
    return ap.parse_args(argv)


# ---- host CPU ----------------------------------------------------------------------

def cpu_info() -> dict:
    """Usable host cores: the affinity mask, capped by the cgroup CPU quota (the
    GPU box shows 256 CPUs but grants 16 through cpu.max)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    usable = max(1, min(aff, int(quota)) if quota else aff)
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"usable": usable, "affinity": aff, "cgroup_quota": quota, "os_cpu_count": os.cpu_count(), "model": model}


# ---- launcher ----------------------------------------------------------------------

def spawn_ranks(args, argv) -> int:
    """`--gpus N` without a torch.distributed environment: run N ranks as a child
    torch.distributed.run (no GPU has been touched in this process)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# ---- the oracle leg (checker + CPU baseline) ---------------------------------------

class OracleChecker:
    """Recomputes gates of the timed batch on the host with the CPU oracle
    (test infrastructure, oracle/): the checker of the run and, at N = 1, the
    CPU baseline.  Never on the measured path."""

    kind = "port"

    def __init__(self, p, lwe: bool):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle
        pyoracle.build()
        self.po = pyoracle
        self.p, self.lwe = p, lwe
        m = pyoracle.XZW_B if p.method != 0 else pyoracle.XZW
        # MK-LWE's accumulator exponents are already mod 2N (ModSwitch in the head)
        q = 2 * p.N if lwe else p.q
        self.orc = pyoracle.Oracle(m, p.k, p.n, p.N, p.Q, q, p.baseG, p.digitsG, p.root)

    def evalacc(self, evk, pkey, ct, acc, threads):
        return self.orc.evalacc_batch(evk, pkey, ct, acc, threads)

    def gates(self, keys, ksk, inputs, threads, ks):
        """Full NAND gates (head, EvalAcc, tail) of the gates in `inputs`."""
        from concurrent.futures import ThreadPoolExecutor
        po, orc, p = self.po, self.orc, self.p
        qKS, baseKS, n_out = ks
        evk, pkey = keys
        G = inputs["a1"].shape[0]
        if self.lwe:
            heads = [orc.mklwe_head(inputs["a1"][g], inputs["b1"][g], inputs["a2"][g], inputs["b2"][g], p.q)
                     for g in range(G)]
            ct = np.stack([h[0] for h in heads])
            acc0 = np.stack([h[1] for h in heads])
        else:
            ct = np.stack([po.mntru_head(inputs["nand"], inputs["a1"][g], inputs["a2"][g], p.q) for g in range(G)])
            acc0 = np.broadcast_to(orc.mntru_testvector(4), (G, p.k, p.N)).copy()
        acc = orc.evalacc_batch(evk, pkey, ct, acc0, threads)
        if self.lwe:
            A, Bk = ksk
            tail = lambda g: orc.mklwe_tail(acc[g], A, Bk, qKS, baseKS, n_out)   # noqa: E731
        else:
            tail = lambda g: orc.mntru_tail_ksk1(acc[g], ksk, qKS, baseKS, n_out)   # noqa: E731
        with ThreadPoolExecutor(max(1, threads)) as ex:   # ctypes releases the GIL
            outs = list(ex.map(tail, range(G)))
        if self.lwe:
            return np.stack([o[0] for o in outs]), np.array([o[1] for o in outs], dtype=np.uint64)
        return np.stack(outs), None


# ---- one rank ----------------------------------------------------------------------

def run_rank(args, env: dict, make_engine, make_checker, torch_device: str, backend: str) -> dict | None:
    """Bench logic of one rank: key broadcast + device upload, this rank's shard
    of synthetic gates, warmup, barrier-bracketed timing of K steps, max over
    ranks, the oracle check of G gates spread over the timed batch, and (rank 0)
    the JSON result.  make_engine / make_checker / torch_device / backend are
    the only things tests/test_bench_ranks.py replaces (CPU stand-ins, gloo)."""
    import torch
    import torch.distributed as dist

    from mkfhe_amd import shard

    world, rank = int(env.get("WORLD_SIZE", 1)), int(env.get("RANK", 0))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1:
        dist.init_process_group(backend, rank=rank, world_size=world, timeout=datetime.timedelta(minutes=10))
    is_cuda = torch_device.startswith("cuda")

    def sync_dev():
        if is_cuda:
            torch.cuda.synchronize()

    eng = make_engine()
    p = eng.params
    wide = eng.wide
    word = 8 if p.Q > (1 << 32) else 4
    B = args.batch
    lwe = p.method != 0
    stage = "evalacc" if wide else args.stage
    qKS, baseKS, n_out = p.q, 32, p.n          # modKS = mod, baseKS = 32 in every MK set (binfhecontext.cpp:129-144)
    dks = int(np.ceil(np.log(qKS) / np.log(baseKS)))

    # ---- keys: drawn on rank 0, broadcast once (RCCL over xGMI), uploaded from the device buffer ----
    # dist.broadcast on NCCL only orders torch's current stream; the engine converts the
    # keys on its own stream, so the host waits for the received buffer first
    evk_n, pkey_n = int(np.prod(eng.evk_shape)), int(np.prod(eng.pkey_shape))
    bcast = (evk_n + pkey_n) * word          # bytes rank 0 broadcasts (keys), + key-switching keys below
    keys = shard.broadcast_keys(evk_n + pkey_n, p.Q, seed=12345, device=torch_device)
    sync_dev()
    eng.upload_keys_device(keys[:evk_n], keys[evk_n:])
    ksk_d = None
    if stage == "gate":
        if lwe:
            na, nb = p.k * p.N * baseKS * dks * n_out, p.k * p.N * baseKS * dks
            bcast += (na + nb) * 4
            ksk_d = shard.broadcast_keys(na + nb, qKS, seed=23456, device=torch_device)
            sync_dev()
            eng.upload_ksk_device(qKS, baseKS, n_out, d_A=ksk_d[:na], d_B=ksk_d[na:])
        else:
            bcast += p.k * p.N * dks * n_out * 4
            ksk_d = shard.broadcast_keys(p.k * p.N * dks * n_out, qKS, seed=23456, device=torch_device)
            sync_dev()
            eng.upload_ksk_device(qKS, baseKS, n_out, d_ksk=ksk_d)

    # ---- this rank's shard of synthetic gates, resident in device memory ----
    rng = np.random.Generator(np.random.PCG64(1000 + rank))

    def dev_words(a):
        a = np.ascontiguousarray(a)
        if a.dtype == np.uint64:
            return torch.from_numpy(a.view(np.int64)).to(torch_device)
        return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).to(torch_device)

    kn = p.k * p.n
    if stage == "gate":
        h = {"a1": rng.integers(0, p.q, size=(B, p.k, p.n), dtype=np.uint32),
             "a2": rng.integers(0, p.q, size=(B, p.k, p.n), dtype=np.uint32),
             "nand": rng.integers(0, p.q, size=(p.k, p.n), dtype=np.uint32)}
        if lwe:
            h["b1"] = rng.integers(0, p.q, size=B, dtype=np.uint32)
            h["b2"] = rng.integers(0, p.q, size=B, dtype=np.uint32)
        d = {key: dev_words(v) for key, v in h.items()}
        d_oa = torch.empty((B, p.k, n_out), dtype=torch.int32, device=torch_device)
        d_ob = torch.empty(B, dtype=torch.int32, device=torch_device) if lwe else None

        def run_step():
            eng.eval_nand_device(d["nand"], d["a1"], d.get("b1"), d["a2"], d.get("b2"), d_oa, d_ob, B)
    else:
        ct_h, acc_h = shard.synthetic_gates(eng, B, seed=1000 + rank)
        d_ct, d_in = dev_words(ct_h), dev_words(acc_h)
        d_out = torch.empty_like(d_in)

        def run_step():
            eng.eval_batch_device(d_ct, d_in, d_out, B)

    # ---- timed region: barrier + sync on both sides, max over ranks ----
    for _ in range(args.warmup):
        run_step()
    eng.sync()
    sync_dev()
    if world > 1:
        dist.barrier()
    sync_dev()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run_step()
    eng.sync()          # also raises on a device-side input-range error
    sync_dev()
    if world > 1:
        dist.barrier()
    sync_dev()
    wall = time.perf_counter() - t0
    elapsed = torch.tensor([wall], dtype=torch.float64, device=torch_device)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    T = float(elapsed.item())

    # ---- dominant kernel (the accumulator step), timed live with HIP events on
    # the engine stream: one EvalAcc pass = k*n step launches (+2 tiny kernels)
    per_launch_s = None
    if is_cuda:
        ct2, acc2 = shard.synthetic_gates(eng, B, seed=2000 + rank)
        e_ct, e_in = dev_words(ct2), dev_words(acc2)
        e_out = torch.empty_like(e_in)
        stream = torch.cuda.ExternalStream(eng.stream_handle())
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        eng.eval_batch_device(e_ct, e_in, e_out, B)
        ev1.record(stream)
        eng.sync()
        per_launch_s = ev0.elapsed_time(ev1) / 1e3 / (p.k * p.n)
        del e_ct, e_in, e_out

    # ---- proof: G gates of this rank's timed batch against the oracle, spread over
    # the whole batch (first and last gate included, so every workgroup slot
    # and dispatch round is sampled -- a first-G sample once hid a defect that
    # only hit gates from the second workgroup slot of each CU) ----
    cpu = cpu_info()
    G = args.check_gates or (cpu["usable"] if world == 1 else 2)
    G = max(1, min(G, B))
    idx = np.unique(np.round(np.linspace(0, B - 1, G)).astype(np.int64))
    G = len(idx)
    threads = args.cpu_threads or (cpu["usable"] if world == 1 else max(1, min(G, cpu["usable"] // world)))
    chk = make_checker(p, lwe)
    keys_h = keys.cpu().numpy().view(np.uint64 if word == 8 else np.uint32)
    evk_h = keys_h[:evk_n].astype(np.uint64).reshape(eng.evk_shape)
    pkey_h = keys_h[evk_n:].astype(np.uint64).reshape(eng.pkey_shape)
    del keys
    if stage == "gate":
        ksk_h = ksk_d.cpu().numpy().view(np.uint32)   # the checker's host copy, after the timed region
        del ksk_d
        ksk64 = ((ksk_h[:na].astype(np.uint64), ksk_h[na:].astype(np.uint64)) if lwe else ksk_h)

    def check(idx):
        """oracle recomputation of gates idx of the timed batch: (mismatch per gate, wall s)"""
        idx_d = torch.as_tensor(idx, device=torch_device)
        n = len(idx)
        t_c = time.perf_counter()
        if stage == "gate":
            sub = {key: (v[idx] if key != "nand" else v) for key, v in h.items()}
            exp_a, exp_b = chk.gates((evk_h, pkey_h), ksk64, sub, threads, (qKS, baseKS, n_out))
            dt = time.perf_counter() - t_c
            got_a = d_oa[idx_d].cpu().numpy().view(np.uint32).astype(np.uint64)
            bad = np.any((got_a != exp_a.reshape(got_a.shape)).reshape(n, -1), axis=1)
            if lwe:
                bad |= d_ob[idx_d].cpu().numpy().view(np.uint32).astype(np.uint64) != exp_b
        else:
            exp = chk.evalacc(evk_h, pkey_h, ct_h[idx].astype(np.uint64), acc_h[idx].astype(np.uint64), threads)
            dt = time.perf_counter() - t_c
            got = d_out[idx_d].cpu().numpy().view(np.uint64 if word == 8 else np.uint32).astype(np.uint64)
            bad = np.any((got != exp).reshape(n, -1), axis=1)
        return bad, dt

    bad, dt_c = check(idx)
    # the CPU baseline's sample: at N = 1 more gates of the batch (evenly spread, not yet
    # checked) until the oracle has done about --cpu-seconds of CPU work (threads x wall);
    # they are parity-checked too
    if world == 1 and args.cpu_baseline and not args.check_gates and G < B and dt_c > 0:
        per_gate_cpu = dt_c * threads / G
        more = int(np.ceil(max(0.0, args.cpu_seconds - dt_c * threads) / per_gate_cpu / threads)) * threads
        more = min(more, B - G, 64 * threads)
        if more > 0:
            rest = np.setdiff1d(np.arange(B, dtype=np.int64), idx)
            idx2 = rest[np.unique(np.round(np.linspace(0, len(rest) - 1, more)).astype(np.int64))]
            bad2, dt2 = check(idx2)
            bad, dt_c, G = np.concatenate([bad, bad2]), dt_c + dt2, G + len(idx2)
    counts = torch.tensor([G, int(bad.sum())], dtype=torch.int64, device=torch_device)
    if world > 1:
        dist.all_reduce(counts, op=dist.ReduceOp.SUM)
    checked, mismatches = int(counts[0].item()), int(counts[1].item())
    # what every rank did: its gates of the global batch (contiguous, B per GPU), the oracle
    # threads of its check and what it checked (tests/test_bench_ranks.py asserts them)
    mine = {"rank": rank, "gates": list(shard.shard_range(world * B, rank, world)), "oracle_threads": threads,
            "checked": G, "mismatches": int(bad.sum()), "keys_received_bytes": bcast}
    ranks = [None] * world
    if world > 1:
        dist.all_gather_object(ranks, mine)
    else:
        ranks = [mine]

    result = None
    if rank == 0:
        dg = p.digitsG - 1
        nk = 1 if lwe else 2
        mm, by = algorithmic_counts(p.k, p.n, dg, nk, p.N, B, word)
        stage_txt = ("NAND gates: head + BootstrapGateCore (EvalAcc) + extraction/ModSwitch/"
                     f"{'KeySwitch' if lwe else 'KeySwitch2'}") if stage == "gate" else "EvalAcc (blind rotation) only"
        pl = per_launch_s or float("nan")
        wide_fp = wide and getattr(eng, "wide_fp", False)
        kname = eng.step_kernel_name(B) if hasattr(eng, "step_kernel_name") else "mk_step_kernel"
        # the engine cuts a batch of >= 2 units of (CUs x 4) gates into MKACC_STREAMS (default 2)
        # slices whose step launches run concurrently on streams of their own
        # (mkacc_engine.hip launch_steps / wide_launch_batch): one accumulator step of the
        # batch is then `slices` launches, and per_launch_us is the time of one such step
        slices = 1
        if is_cuda and kname in ("mk_step_kernel", "mk_step2_kernel", "widereg2::step_kernel"):
            import torch
            cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
            ev = os.environ.get("MKACC_STREAMS", "")
            slices = max(1, min(int(ev) if ev in ("1", "2", "3", "4") else 2, B // (cus * 4)))
        traffic = (measured_traffic(args.paramset + ("_q50" if args.q_bits == 50 else ""), kname, by)
                   if not args.n_override else {"bytes": None, "why": "--n-override"})
        peak_mm, peak_src = ((PEAK_FP64_MULMOD_TPS, "exact FP64 product, profiles/r2/ubench_wide.txt") if wide_fp else
                             (PEAK_INT64_MULMOD_TPS, "64-bit Shoup product, profiles/r2/ubench_wide.txt") if wide else
                             (PEAK_SHOUP_MULMOD_TPS, "27-bit Shoup product, profiles/round1_ubench_intops.txt"))
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
            "dtype": ("f64 (exact integer residues mod a 50-bit Q; u64 words at the boundary)" if wide_fp else
                      "u64 (residues mod Q)") if word == 8 else "u32 (27-bit residues mod Q)",
            "data": "synthetic: uniform keys, key-switching keys and ciphertexts (seeded)",
            "config": {"workload": f"{args.paramset} {p.k}-party {'MK-LWE' if lwe else 'MK-NTRU'} {stage_txt} "
                                   f"(k={p.k}, n={p.n}, N={p.N}, dg={dg}"
                                   + (f", Q={p.Q} in 64-bit words, B_g=2^{p.baseG.bit_length() - 1})" if wide else ")"),
                       "paramset": args.paramset, "stage": stage, "batch_per_gpu": B, "global_batch": world * B,
                       "parallelism": f"gate-sharded x{world}" + (" (rehearsal: every rank on one GPU, gloo)"
                                                                   if getattr(args, "shared_gpu", False) else "")},
            "parity_checked": checked,
            "parity_mismatches": mismatches,
            "keys_broadcast_bytes": bcast,
            "ranks": ranks,
            "parity": (f"{G} gates of every rank's timed batch, evenly spread from the first to the last, "
                       "recomputed by the CPU oracle (oracle/, "
                       "bit-exact integer compare of every output word); the oracle's primitives are pinned by the "
                       "reference's KATs, the EvalAcc composition is 'parity unpinned' beyond them (DESIGN.md s3)"),
            "roofline": {"bound": "hbm", "achieved": by / pl / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": by / pl / 1e9 / PEAK_HBM_GBS,
                         "traffic": traffic["bytes"],
                         "traffic_record": traffic,
                         "kernel": kname,
                         "per_launch_us": pl * 1e6,
                         "bytes_per_launch": by,
                         "slices_per_step": slices,
                         "launch_note": ("one accumulator step of the whole batch: " + (
                             f"{slices} concurrent launches of {B // slices}+ gates on {slices} streams; rocprof lists each "
                             "slice launch with its own (overlapping) duration" if slices > 1 else
                             "the pass time / (k n): small batches run the steps after the first in one launch "
                             "(mk_quadp_run_kernel at B <= CUs / 2, mk_quad_run_kernel at B <= CUs, mk_quad2_run_kernel "
                             "up to 4 gates per CU, DESIGN.md s2)"
                             if kname in ("mk_lat_kernel", "mk_latd_kernel", "mk_lat_run_kernel", "mk_latd_run_kernel",
                                          "mk_quad_kernel", "mk_quad_run_kernel", "mk_quad2_kernel",
                                          "mk_quad2_run_kernel", "mk_quadp_run_kernel")
                             else "one launch"))},
            # VALU view: algorithmic mod-muls per launch against the measured rate of the
            # product the kernel is built on (32-bit Shoup; FP64 or 64-bit Shoup on the wide path)
            "roofline_valu": {
                "bound": "valu-fp64" if wide_fp else "valu-int", "achieved": mm / pl / 1e12,
                "peak": peak_mm / 1e12, "unit": "T mod-mul/s", "frac": mm / pl / peak_mm,
                "mulmods_per_launch": mm, "peak_source": peak_src},
        }
        if world == 1 and args.cpu_baseline:
            what = ("NAND gates (head + EvalAcc + extraction/ModSwitch/key switch)" if stage == "gate"
                    else "EvalAccs")
            ref = REF_CPU_S_PER_EVALACC.get(args.paramset) if not (wide or args.n_override) else None
            o_r = oracle_over_ref()
            result["cpu_baseline"] = {
                "value": G / dt_c, "unit": "bootstraps/s", "cores": threads, "kind": chk.kind,
                "sample": (f"{G} {what} spread over the timed batch ({p.k}x{p.n} accumulator steps each), one per "
                           f"thread at a time on {threads} threads, {dt_c:.2f} s wall ({dt_c * threads:.1f} thread-s); the same gates "
                           "are the parity check"),
                "host": cpu,
                "reference_1core_s_per_evalacc": ref,
                "oracle_over_reference_1core": o_r.get(args.paramset) if ref else None,
                # the reference's throughput on the same cores, scaled by the 1-core time ratio:
                # an estimate (the ratio compares two different CPUs, calibration()); only
                # "value" above is measured on this box
                "reference_equivalent_estimate": (G / dt_c * o_r[args.paramset]
                                                  if ref and args.paramset in o_r else None),
                "calibration": calibration() if ref else None,
                "reference_source": "SURVEY.md s6: the reference's own EvalAcc, 1 thread of the survey container",
            }
    if world > 1:
        dist.destroy_process_group()
    if mismatches:
        if rank == 0:
            print(json.dumps(result), flush=True)
        raise SystemExit(f"parity FAILED: {mismatches} of {checked} checked gates differ from the oracle")
    return result


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args, argv))
    env = dict(os.environ)
    local = int(env.get("LOCAL_RANK", "0"))

    if args.stub_engine:   # CPU rehearsal of the rank logic (tests/test_bench_ranks.py)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import bench_stub
        res = run_rank(args, env, lambda: bench_stub.StubEngine(args), bench_stub.StubChecker, "cpu", "gloo")
    else:
        import torch
        import mkfhe_amd as mk

        dev = 0 if args.shared_gpu else local
        torch.cuda.set_device(dev)

        def make_engine():
            p = mk.paramset(args.paramset)
            if args.n_override:
                p.n = args.n_override
            if args.q_bits == 50:   # SURVEY.md s8 config 5 stress (s6: reference CPU 0.568 s / EvalAcc at k=2, n=560)
                p.Q, p.baseG, p.digitsG, p.root = Q50, 1 << 10, 0, 0
            return mk.MKAccumulatorEngine(p, device=dev)

        res = run_rank(args, env, make_engine, OracleChecker, f"cuda:{dev}", "gloo" if args.shared_gpu else "nccl")
    if res is not None:
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
