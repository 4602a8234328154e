#!/usr/bin/env python3
"""Throughput of the MI355X Bussgang-GMM estimate path (BASELINE.json metric).

A step is one ``estimate_from_y`` of the reference (gmm_cplx_bussgang.py:166-243) over one batch:
the per-SNR FP64 precompute (prepare) followed by the fused estimate kernel, with the batch of
quantised observations already resident in HBM.  Default workload = the metric configuration
(SURVEY.md §8(d) D2): K=128 components, N=M=64 antennas, 'full' covariances, 1-bit uniform
quantiser, SNR 5 dB, mode 'all', B=100,000 observations, FP64 arithmetic (the reference's complex128).

  python bench.py [--gpus N --steps K --warmup W] [--config metric|cfg1..cfg5|cfg3dense|cfg5dense]
                  [--shard batch|k] [--precision f64|fast] [--chunks C]

Multi-GPU: one process per GPU.  ``--gpus N`` without a torch.distributed launcher starts the N ranks
itself (child processes, before any GPU call); under ``torch.distributed.run`` the ranks come from the
environment and must number ``--gpus``.  ``--shard k`` (default for the dense configs: metric, cfg1,
cfg2, cfg4) splits the K components over the ranks (strong scaling: the B observations are estimated
once by the whole node) and sums the shifted FP64 partials with one RCCL reduce-scatter per batch
chunk, pipelined behind the next chunk's kernel; ``--shard batch`` (default for the
Fourier paths cfg3 / cfg5) gives every rank its own B observations and the whole mixture (no
data-path collective, weak scaling).  Rank 0 prints one JSON line.
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "channel estimates/sec + MSE vs reference; K=128 N=64 full-cov, 1/2/4/8 GPU"
FP64_MFMA_PEAK_TFLOPS = 78.6  # MI355X_MICROARCH.md / SURVEY D3: v_mfma_f64_16x16x4_f64 dense peak (spec)
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak (spec)
FP16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense FP16/BF16 MFMA (spec, no sparsity)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec (6.3 TB/s measured copy)

CONFIGS = {
    "metric": dict(K=128, N=64, cov="full", n_bits=1, qtype="uniform", B=100_000, snr=5.0),
    "cfg1": dict(K=16, N=32, cov="full", n_bits=1, qtype="uniform", B=1_000, snr=5.0),
    "cfg2": dict(K=64, N=64, cov="full", n_bits=1, qtype="uniform", B=10_000, snr=5.0),
    "cfg3": dict(K=128, N=64, cov="circulant", n_bits=3, qtype="lloyd", B=100_000, snr=5.0),
    "cfg3dense": dict(K=128, N=64, cov="circulant", n_bits=3, qtype="lloyd", B=100_000, snr=5.0, dense=True),
    "cfg4": dict(K=256, N=128, cov="full", n_bits=1, qtype="uniform", B=50_000, snr=5.0),
    "cfg5": dict(K=128, N=256, cov="block-circulant", blocks=(4, 64), n_bits=2, qtype="uniform", B=100_000,
                 snr=5.0),
    "cfg5dense": dict(K=128, N=256, cov="block-circulant", blocks=(4, 64), n_bits=2, qtype="uniform", B=100_000,
                      snr=5.0, dense=True),
}
DEFAULT_SHARD = {"metric": "k", "cfg1": "k", "cfg2": "k", "cfg4": "k", "cfg3": "batch", "cfg3dense": "batch",
                 "cfg5": "batch", "cfg5dense": "batch"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="metric", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0, help="override B (observations per step)")
    ap.add_argument("--components", type=int, default=0, help="override K (PMC calibration runs)")
    ap.add_argument("--shard", default=None, choices=["batch", "k"])
    ap.add_argument("--precision", default="f64", choices=["f64", "fast"],
                    help="dense 'all' arithmetic: f64 (the reference's complex128, default) or fast (fp16 split)")
    ap.add_argument("--chunks", type=int, default=0,
                    help="K-shard pipeline chunks per batch (0 = sharding.default_chunks: 2)")
    ap.add_argument("--backend", default="native",
                    help="K-shard collectives: native (libqce's own RCCL communicator, qce_kshard_*; torch.distributed "
                         "over gloo only for the rendezvous, barriers and the timing MAX) or a torch.distributed "
                         "backend (nccl = RCCL through torch, gloo) driving sharding.py's Python orchestration")
    ap.add_argument("--comm", default="auto", choices=["auto", "rccl", "host"],
                    help="native K-shard communicator: rccl (ncclCommInitRank, one GPU per rank), host (the library's "
                         "host transport over gloo: ranks may share a GPU) or auto (host when the ranks outnumber the "
                         "visible GPUs -- the one-GPU rehearsal of the driver's multi-GPU command -- else rccl)")
    ap.add_argument("--collective", default="rs", choices=["rs", "ar"],
                    help="K-shard SUM collective: reduce-scatter (rank keeps its rows) or all-reduce")
    ap.add_argument("--single-buffer", action="store_true",
                    help="native K-shard: one table set (no overlap of the next prepare with the current step)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU-baseline budget per leg (0 = skip)")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the fast-path side line")
    ap.add_argument("--dropin", action="store_true",
                    help="add the drop-in (numpy host I/O) side line; off by default because its chunked launches of "
                         "the headline kernel would enter a rocprof kernel-stats average of the bench command")
    ap.add_argument("--mean", action="store_true",
                    help="components with non-zero means (0.3 x CN(0, 1) per entry, seeded): the reference's fit "
                         "default zero_mean=False (gmm_cplx_bussgang.py:96-100); the bench configs are zero-mean")
    ap.add_argument("--sweep", action="store_true",
                    help="one GPU: the reference's SNR loop (Bussgang_GMM.py:43, :284-287: snrs -10..20 dB, one batch "
                         "of B observations per point) with double-buffered per-SNR tables (sweep.SnrSweep: the prepare "
                         "of point t+1 beside the estimate of point t), against the same loop prepare-then-estimate")
    ap.add_argument("--launch-check", action="store_true",
                    help="CPU rehearsal of the launcher: ranks rendezvous over gloo, barrier + MAX-over-ranks "
                         "timing, rank 0 prints one JSON line; no GPU is touched")
    ap.add_argument("--traffic", default=None,
                    help="JSON with PMC-derived HBM bytes per launch of the estimate kernel "
                         "(default profiles/traffic_<config>.json, traffic_<config>_mean.json with --mean)")
    a = ap.parse_args()
    if a.shard is None:
        a.shard = DEFAULT_SHARD[a.config]
    return a


# ------------------------------------------------------------------------------------------ launcher
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n):
    """Start n ranks of this script (one per GPU) before anything touches the GPU; exit with the worst
    status.  A rank that fails takes the others down (their PIDs, not a pattern)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0:
                rc = rc or c
                for q in live:
                    q.kill()
        time.sleep(0.05)
    return rc


def launch_check(args):
    """The multi-rank skeleton of main() without a GPU: rendezvous, barrier, per-rank timing reduced with
    MAX, one JSON line from rank 0 (tests/test_sharding_cpu.py runs it at world size 2 over gloo)."""
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
    elapsed = 0.01 * (rank + 1)
    t = torch.tensor([elapsed, float(rank)], dtype=torch.float64)
    ranks = [rank]
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        out = [None] * world
        dist.all_gather_object(out, rank)
        ranks = out
        dist.barrier()
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": args.gpus, "world_size": world, "ranks": ranks,
                          "max_elapsed": float(t[0])}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


# ------------------------------------------------------------------------------------------ inputs
def make_inputs(cfg, seed, pool=2048):
    """Synthetic batch of the configured shape: SCM channels (a seeded pool of `pool` distinct
    channels, reused with fresh noise) -> quantised observations y = Q(h + n)."""
    from quantized_channel_estimation_amd import inputs
    K, N, B = cfg["K"], cfg["N"], cfg["B"]
    means, covs, w = inputs.synthetic_model(K, N, cov_type=cfg["cov"], blocks=cfg.get("blocks"))
    if cfg.get("mean"):
        means = 0.3 * inputs.crandn(K, N, rng=np.random.default_rng(12))
    rng = np.random.default_rng(1000 + seed)
    hp, _ = inputs.scm_generate(min(pool, B), 1, N, rng, n_path=3)
    hp = hp[:, 0, :].astype(np.complex128)
    h = hp[rng.integers(0, hp.shape[0], size=B)]
    quantizer = (None, None, None)
    if cfg["n_bits"] not in (1, np.inf):
        quantizer = inputs.get_quantizer([cfg["snr"]], cfg["n_bits"], cfg["qtype"])[cfg["snr"]]
    y = inputs.get_observation_nbit(h, cfg["snr"], None, cfg["n_bits"], quantizer[0], quantizer[1],
                                    rng=np.random.default_rng(2000 + seed))
    return means, covs, w, h, np.ascontiguousarray(y, dtype=np.complex128), quantizer


# ------------------------------------------------------------------------------------------ CPU baseline
def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def available_cpus():
    """CPUs this process may actually use: the affinity mask, capped by a cgroup (v2 cpu.max / v1 cfs) CPU quota
    when one is set.  Returns (count, basis)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0 and per > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    n, basis = aff, f"sched_getaffinity {aff}"
    if quota is not None and quota < n:
        n, basis = max(1, int(quota)), f"cgroup CPU quota {quota:g} (affinity {aff})"
    # the host's declared CPU share per GPU job (the GPU box exports OMP_NUM_THREADS = its share)
    share = os.environ.get("OMP_NUM_THREADS", "")
    if share.isdigit() and 0 < int(share) < n:
        n, basis = int(share), f"OMP_NUM_THREADS {share} = the job's CPU share (affinity {aff}, quota {quota})"
    return n, basis + f"; nproc {os.cpu_count()}"


def _pool_worker(args):
    """One Pool worker: the loop-faithful oracle on its shard, single-threaded BLAS (the reference's
    mp_gmm worker, Bussgang_GMM.py:16-17, one estimate_from_y per task incl. its prepare)."""
    from threadpoolctl import threadpool_limits
    from oracle import qce_oracle as O
    means, covs, w, y, snr, N, n_bits, qtype, quantizer = args
    with threadpool_limits(limits=1):
        t0 = time.perf_counter()
        O.estimate_loop(means, covs, w, y, snr, N, None, n_bits, qtype, quantizer)
        return time.perf_counter() - t0


def cpu_baseline(cfg, means, covs, w, y, quantizer, budget_s):
    """The reference's CPU path timed on this host: the loop-faithful restatement
    (same per-(sample, component) op order as gmm_cplx_bussgang.py:223-228 incl. the redundant
    C_k A_eff^H) (i) in one process, one BLAS thread, (ii) in a Pool of single-thread workers sharding the
    batch, sized as Bussgang_GMM.py:29-32 sizes its pool (cpu_count()//2) from the CPUs this process can
    actually use (affinity mask and cgroup quota, measured: available_cpus), and (iii) the vectorised FP64
    oracle ("optimised CPU", BLAS threads = the pool size).  Bounded samples: the cost is linear in B
    (per-call prepare included)."""
    import multiprocessing as mp
    from threadpoolctl import threadpool_limits
    from oracle import qce_oracle as O
    N, snr, nb, qt = cfg["N"], cfg["snr"], cfg["n_bits"], cfg["qtype"]
    nproc = os.cpu_count() or 1
    avail, basis = available_cpus()
    npool = max(1, avail // 2)

    def loop(n):
        t0 = time.perf_counter()
        O.estimate_loop(means, covs, w, y[:n], snr, N, None, nb, qt, quantizer)
        return time.perf_counter() - t0

    with threadpool_limits(limits=1):
        a, b = (4, 24) if N <= 64 else (1, 3)
        t1, t2 = loop(a), loop(b)
        per = max((t2 - t1) / (b - a), 1e-6)
        prep = max(t1 - a * per, 0.0)
        n1 = int(max(b, min(y.shape[0], (budget_s - prep) / per)))
        dt1 = loop(n1)
    single = dict(value=round(n1 / dt1, 2), cores=1, sample=f"{n1} observations, {dt1:.1f} s (prepare included)")
    # (ii) process pool, one shard per worker
    nper = int(max(2, min(y.shape[0] // npool, (budget_s - prep) / per)))
    tasks = [(means, covs, w, y[i * nper:(i + 1) * nper], snr, N, nb, qt, quantizer) for i in range(npool)]
    ctx = mp.get_context("fork")
    pool = ctx.Pool(npool)
    try:
        t0 = time.perf_counter()
        pool.map(_pool_worker, tasks, chunksize=1)
        dtp = time.perf_counter() - t0
        pool.close()  # workers exit on their own (Pool.__exit__ would terminate() them with SIGTERM)
    finally:
        pool.join()
    pooled = npool * nper / dtp
    # (iii) vectorised oracle
    with threadpool_limits(limits=npool):
        nv = min(y.shape[0], 2000 if N <= 64 else 400)
        t0 = time.perf_counter()
        O.estimate(means, covs, w, y[:nv], snr, N, None, "all", nb, qt, quantizer)
        dtv = time.perf_counter() - t0
    return dict(value=round(pooled, 2), unit="channel estimates/s", cores=npool, kind="port",
                sample=f"Pool({npool}) of single-thread workers (Bussgang_GMM.py:29-32 sizing: available CPUs // 2), "
                       f"{nper} observations each through oracle.estimate_loop (per-call prepare included), "
                       f"{dtp:.1f} s wall",
                nproc=nproc, cpus_available=avail, cpus_basis=basis, cpu_model=_cpu_model(), single_process=single,
                vectorised=dict(value=round(nv / dtv, 2), cores=npool,
                                sample=f"{nv} observations through oracle.estimate (vectorised FP64), {dtv:.2f} s"))


# ------------------------------------------------------------------------------------------ roofline
def f64_executed_flops(N, K, B):
    """Executed v_mfma_f64_16x16x4 work of k_est_all_f64: 256 flops per sample per 1 KB table block
    (GL: NTL(NTL+1) blocks — Linv's upper triangle skipped; GW: NTW*KP blocks).  At padded 128 the row-split wave
    pairs pad each GL tile pair to 4j + 4 k-pairs per half (qce_f64_kernel.h f64_pr): 4 J (J + 1) GL blocks, J = NTL / 2."""
    Np = 16 if N <= 16 else (32 if N <= 32 else (64 if N <= 64 else 128))
    ntl, ntw, kp = Np // 8, Np // 8, Np // 4
    gl = ntl * (ntl + 1)
    if Np == 128:  # pairs: virtual tile j (4j + 4 k-pairs) executed by both halves
        J = ntl // 2
        gl = 2 * sum(4 * j + 4 for j in range(J))
    return 256.0 * (gl + ntw * kp) * K * B


def f64g_executed_flops(N, K, B, has_mean=False):
    """Executed v_mfma_f64_16x16x4 work of k_est_all_f64g (3M): per component and 16 samples 6 MFMAs per unit of two
    k-steps and 16-row tile -- GL: 2T + 2 units for tile T (the 16-row triangle), GW: MP / 8 units per tile -- plus
    2 per tile for the mean / bias columns; 2048 flops per MFMA over 16 samples."""
    if N > 64:
        # k_est_all_f64h (padded 128, row halves): per half 3 blocks per GL unit (36 units; + a 3-block mean unit per
        # tile with means) and 192 GW blocks (+ 4 bias blocks), two MFMAs per block
        hm = 1 if has_mean else 0
        mf = 2 * (2 * 3 * (36 + 4 * hm) + 2 * (192 + 4 * hm))
        return 2048.0 / 16.0 * mf * K * B
    Np = 16 if N <= 16 else (32 if N <= 32 else 64)
    ntl = ntw = Np // 16
    mf = 6 * sum(2 * t + 2 for t in range(ntl)) + 6 * (Np // 8) * ntw + (2 * (ntl + ntw) if has_mean else 0)
    return 2048.0 / 16.0 * mf * K * B


def dm_has_mean(dm):
    """Whether the device model carries non-zero means (the bench's synthetic models are zero-mean)."""
    return bool(getattr(dm, "has_mean", False))


def roofline_line(args, cfg, dm, k_local, B, kern_ms, traffic):
    N = cfg["N"]
    fourier = bool(dm.structure()[2])
    if fourier:
        # HBM-bound: 16 M bytes of y in + 16 N bytes of h out per estimate (c128)
        bytes_per_launch = 32.0 * N * B
        achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
        n1, n2, _ = dm.structure()
        # D3: 4 K N MFMA flops per estimate (zero mean; 12 K N with means: + 2 Re(Y^* u) in lp, + b in the filter)
        fft_flops = ((12.0 if dm_has_mean(dm) else 4.0) * k_local * N + 10.0 * N * math.log2(N)) * B
        return dict(bound="hbm", achieved=round(achieved, 2), peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=round(achieved / HBM_PEAK_GBS, 4), traffic=traffic,
                    kernel=fourier_kernel(N, dm_has_mean(dm)),
                    structure=f"block-circulant ({n1},{n2})" if n1 > 1 else "circulant",
                    kernel_ms=round(kern_ms, 4), bytes_per_launch=bytes_per_launch,
                    fp64_flops_per_launch=fft_flops, fp64_tflops=round(fft_flops / (kern_ms * 1e-3) / 1e12, 3),
                    fp64_frac=round(fft_flops / (kern_ms * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS, 4),
                    note="HBM roofline per SURVEY D3 (32 N B per estimate); the kernel's binding resource is FP64 "
                         "issue (4 K N MFMA flops per estimate, 12 K N with means, + FFT VALU flops), reported as "
                         "fp64_frac")
    M = N  # A = I at every bench config (n_pilots = 1)
    flops = 16.0 * k_local * N * N * B  # 16 K M N real flops per estimate (dense count)
    if dm.precision == "f64":
        # minimal useful work per (sample, component): the triangular quad form ||Linv y||^2 = M(M+1)/2 complex
        # MACs + the filter W y = M N complex MACs (+ the -q0 and b columns with a mean model).  A complex MAC is
        # 8 real flops as four real products (the 4M kernel, k_est_all_f64) and 6 as Gauss's three (the 3M kernel,
        # k_est_all_f64g): frac counts the flops of the algorithm the kernel runs, so it stays <= 1 either way, and
        # the 4M-equivalent rate (the same work priced at 8 flops per complex MAC) is reported beside it.
        g3 = dm.kernel() == "f64_3m"
        cm = 6.0 if g3 else 8.0
        cmacs = M * (M + 1) / 2.0 + M * N + ((M + N) if dm_has_mean(dm) else 0.0)
        useful_per = cm * cmacs
        useful = useful_per * k_local * B
        achieved = useful / (kern_ms * 1e-3) / 1e12
        frac = achieved / FP64_MFMA_PEAK_TFLOPS
        assert frac <= 1.0, f"roofline frac {frac:.4f} > 1: the useful-work count or the kernel timing is wrong"
        if N > 128:
            kernel = "k_lp_f64 + k_wsum_weights + k_wsum_f64"
        else:
            kernel = (("k_est_all_f64h (3M, row halves)" if N > 64 else "k_est_all_f64g (3M)") if g3
                      else "k_est_all_f64") + " (+k_merge_f64)"
        line = dict(bound="mfma", achieved=round(achieved, 3), peak=FP64_MFMA_PEAK_TFLOPS, unit="TFLOP/s",
                    frac=round(frac, 4), traffic=traffic, kernel=kernel, peak_dtype="fp64 MFMA (dense)",
                    kernel_ms=round(kern_ms, 4), complex_product="3M (Gauss)" if g3 else "4M",
                    useful_flops_per_estimate_component=useful_per,
                    flops_per_launch=useful, dense_16KMN_flops_per_launch=flops,
                    note=("frac = minimal useful flops of the kernel's algorithm (complex MACs of the triangular quad "
                          "form M(M+1)/2 + filter MN, x6 real flops as 3M, x8 as 4M) / kernel time / FP64 MFMA peak; "
                          "mfma_issue_frac = executed MFMA flops / time / peak (the pipe occupancy, includes the "
                          "padding of the 16x16 tiles)"))
        if g3:
            eq = 8.0 * cmacs * k_local * B
            line["equiv_4m_tflops"] = round(eq / (kern_ms * 1e-3) / 1e12, 3)
            line["equiv_4m_frac"] = round(eq / (kern_ms * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS, 4)
        if N <= 128:
            ex = f64g_executed_flops(N, k_local, B, dm_has_mean(dm)) if g3 else f64_executed_flops(N, k_local, B)
            line["executed_flops_per_launch"] = ex
            line["mfma_issue_frac"] = round(ex / (kern_ms * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS, 4)
        return line
    achieved = flops / (kern_ms * 1e-3) / 1e12
    nsl = (2 * N) // 32
    tri = (sum(2 * r + 2 for r in range(nsl)) / (nsl * 2 * nsl) + 1.0) / 2.0
    ex = flops * tri * 2.0
    return dict(bound="mfma", achieved=round(achieved, 3), peak=FP16_MFMA_PEAK_TFLOPS, unit="TFLOP/s",
                frac=round(achieved / FP16_MFMA_PEAK_TFLOPS, 4), traffic=traffic,
                kernel="k_est_all_h2 / k_est_all_h2x", peak_dtype="fp16 MFMA (dense)",
                kernel_ms=round(kern_ms, 4), flops_per_launch=flops,
                mfma_issue_frac=round(ex / (kern_ms * 1e-3) / 1e12 / FP16_MFMA_PEAK_TFLOPS, 4))


def fourier_kernel(N, has_mean):
    """The Fourier-path kernel qce_fft_mfma.hip runs for this shape (QCE_FFT_CHUNK=0 selects the round-2 kernels)."""
    new = os.environ.get("QCE_FFT_CHUNK", "1") != "0"
    if N == 64 and new:
        return "k_fft_wreg<HM>" if has_mean else "k_fft_wreg"
    if N <= 64:
        return "k_fft_wave"
    if not new:
        return "k_fft_mfma"
    return "k_fft_chunk_hm" if has_mean else "k_fft_chunk"


def dtype_of(dm):
    if dm.structure()[2]:
        return "f64"
    if dm.precision == "f64":  # k_est_all_f64 up to padded 128, k_lp_f64 + k_wsum_f64 beyond
        return "f64"
    return "f16x2 (fp16 hi+lo split, fp32 accumulate, fp64 softmax)"


# ------------------------------------------------------------------------------------------ side lines
def fast_line(cfg, means, covs, w, yd, out, stream, steps, qargs, ho, n_chk):
    """The opt-in fast path (fp16 two-term split, fp32 accumulate) on the same workload: its own
    throughput and parity, reported beside the FP64 headline (never as `value`)."""
    import torch
    from quantized_channel_estimation_amd import _lib
    dm = _lib.DeviceModel(means, covs, w)
    dm.set_precision("fast")
    sptr = stream.cuda_stream
    for _ in range(2):
        dm.prepare(None, cfg["snr"], cfg["n_bits"], *qargs, stream=sptr)
        dm.estimate(yd, _lib.MODE_ALL, 0.0, out=out, stream=sptr)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for i in range(steps):
        dm.prepare(None, cfg["snr"], cfg["n_bits"], *qargs, stream=sptr)
        ev[i][0].record(stream)
        dm.estimate(yd, _lib.MODE_ALL, 0.0, out=out, stream=sptr)
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    hg = out[:n_chk].cpu().numpy()
    res = dict(value=round(yd.shape[0] * steps / dt, 1), ms_per_step=round(dt / steps * 1e3, 4),
               kernel_ms=round(kms, 4), dtype=dtype_of(dm))
    if ho is not None:
        res["parity_rel_fro"] = float(np.linalg.norm(hg - ho) / np.linalg.norm(ho))
    dm.close()
    return res


def dropin_line(cfg, means, covs, w, y, quantizer, calls=8):
    """The drop-in API as the scripts call it: Gmm_nbit.estimate_from_y with numpy y in and numpy h out
    (H2D + prepare + kernel + D2H, reference state mirroring deferred until gm is read).  Each call timed on its own
    (the caller's array and the returned one are host memory: a call ends when h is in the numpy array); `value`
    from the median call, the mean beside it."""
    from quantized_channel_estimation_amd import Gmm_nbit
    g = Gmm_nbit.from_params(means, covs, w)
    args = (cfg["snr"], cfg["N"], None, "all", cfg["n_bits"], cfg["qtype"], quantizer)
    for _ in range(2):
        g.estimate_from_y(y, *args)
    ts = []
    for _ in range(calls):
        t0 = time.perf_counter()
        h = g.estimate_from_y(y, *args)
        ts.append(time.perf_counter() - t0)
        del h
    med = float(np.median(ts))
    return dict(value=round(y.shape[0] / med, 1), ms_per_call=round(med * 1e3, 3),
                ms_per_call_mean=round(float(np.mean(ts)) * 1e3, 3), ms_per_call_min=round(min(ts) * 1e3, 3),
                calls=calls, io="host numpy complex128 in/out, state mirror lazy")


# ------------------------------------------------------------------------------------------ SNR sweep
SWEEP_SNRS = [-10, -5, 0, 5, 10, 15, 20]  # Bussgang_GMM.py:43


def sweep_main(args):
    """--sweep: the reference's SNR loop on one GPU, one batch per SNR point, prepare + estimate per point; the
    double-buffered SnrSweep against the serial loop on one model.  One JSON line."""
    import torch
    from quantized_channel_estimation_amd import _lib
    from quantized_channel_estimation_amd.sweep import SnrSweep
    cfg = dict(CONFIGS[args.config])
    if cfg.pop("dense", False):
        os.environ["QCE_FFT"] = "0"
    if args.batch:
        cfg["B"] = args.batch
    K, N, B = cfg["K"], cfg["N"], cfg["B"]
    qkind = {"uniform": _lib.QUANT_UNIFORM, "lloyd": _lib.QUANT_LLOYD}[cfg["qtype"]]
    points_host = []
    for i, snr in enumerate(SWEEP_SNRS):
        c = dict(cfg, snr=float(snr))
        means, covs, w, h, y, qz = make_inputs(c, i)
        thr, lab = (qz[0], qz[1]) if c["n_bits"] not in (1, np.inf) and c["qtype"] == "lloyd" else (None, None)
        points_host.append((float(snr), y, h, qz, thr, lab))
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    pts = [(None, snr, cfg["n_bits"], qkind, thr, lab, torch.from_numpy(y).to(dev))
           for snr, y, h, qz, thr, lab in points_host]
    outs = [torch.empty((B, N), dtype=torch.complex128, device=dev) for _ in pts]
    sw = SnrSweep(means, covs, w, reserve_cus=int(os.environ.get("QCE_SWEEP_RESERVE", "32")))
    single = _lib.DeviceModel(means, covs, w)
    sptr = stream.cuda_stream

    def serial():
        for (A, snr, nb, qk, thr, lab, y), o in zip(pts, outs):
            single.prepare(A, snr, nb, qk, thr, lab, stream=sptr)
            single.estimate(y, _lib.MODE_ALL, 0.0, out=o, stream=sptr)

    def timed(fn):
        for _ in range(max(1, args.warmup)):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / (args.steps * len(pts))

    t_ser = timed(serial)
    ref = [o.cpu().numpy() for o in outs]
    t_dbl = timed(lambda: sw.run(pts, outs=outs, stream=stream))
    got = [o.cpu().numpy() for o in outs]
    dev_vs_serial = max(float(np.linalg.norm(g - r) / np.linalg.norm(r)) for g, r in zip(got, ref))
    parity = None
    if not args.no_parity:
        from oracle import qce_oracle as O
        snr, y, h, qz, thr, lab = points_host[3]
        ho = O.estimate(means, covs, w, y[:512], snr, N, None, "all", cfg["n_bits"], cfg["qtype"], qz)
        parity = dict(snr=snr, samples=512, rel_fro=float(np.linalg.norm(got[3][:512] - ho) / np.linalg.norm(ho)))
    line = {"metric": METRIC + " (SNR sweep)", "value": round(B / t_dbl, 1), "unit": "channel estimates/s",
            "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_snr_point": round(t_dbl * 1e3, 4),
            "ms_per_snr_point_serial": round(t_ser * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic: one seeded batch per SNR point",
            "config": {"workload": f"SNR sweep {SWEEP_SNRS} dB, per point estimate_from_y K={K} N=M={N} "
                                   f"cov={cfg['cov']} n_bits={cfg['n_bits']} {cfg['qtype']} mode=all B={B}",
                       "K": K, "N": N, "B": B, "points": len(pts), "tables": "double-buffered (sweep.SnrSweep)"},
            "kernel": single.kernel(), "max_rel_dev_vs_serial": dev_vs_serial, "parity": parity}
    print(json.dumps(line), flush=True)
    sw.close()
    single.close()
    return 0


# ------------------------------------------------------------------------------------------ main
def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if args.launch_check:
        return launch_check(args)
    if args.sweep:
        if args.gpus != 1:
            raise SystemExit("bench.py --sweep runs on one GPU")
        return sweep_main(args)
    cfg = dict(CONFIGS[args.config])
    if cfg.pop("dense", False):
        os.environ["QCE_FFT"] = "0"  # read by qce_prepare: keep the structured mixture on the dense path
    import torch
    import torch.distributed as dist
    from quantized_channel_estimation_amd import _lib
    from quantized_channel_estimation_amd.sharding import ComponentShardEstimator, component_slices, default_chunks

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    # ranks beyond the visible GPUs share them (single-GPU rehearsals of the multi-rank path; on a node
    # with one GPU per rank this is the identity).  device_count() does not initialise the GPU.
    ndev = torch.cuda.device_count()
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, ndev)
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if args.batch:
        cfg["B"] = args.batch
    if args.components:
        cfg["K"] = args.components
    if args.mean:
        cfg["mean"] = True
    K, N, B = cfg["K"], cfg["N"], cfg["B"]
    data_seed = rank if args.shard == "batch" else 0
    means, covs, w, h, y, quantizer = make_inputs(cfg, data_seed)
    # the CPU baseline runs first, before this process touches the GPU (its Pool forks workers)
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(cfg, means, covs, w, y, quantizer, args.cpu_seconds)
    torch.cuda.set_device(local)
    native = args.backend == "native"
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:  # native: the data path runs on libqce's RCCL communicator; gloo carries the control traffic
            dist.init_process_group("gloo" if native else args.backend)
        world = dist.get_world_size()
    kshard = args.shard == "k" and world > 1
    comm_kind = None
    qkind = {"uniform": _lib.QUANT_UNIFORM, "lloyd": _lib.QUANT_LLOYD}[cfg["qtype"]]
    thr, lab = (quantizer[0], quantizer[1]) if cfg["n_bits"] not in (1, np.inf) and cfg["qtype"] == "lloyd" else \
        (None, None)
    qargs = (qkind, thr, lab)

    dev = torch.device("cuda", local)
    yd = torch.from_numpy(y).to(dev)
    out = torch.empty((B, N), dtype=torch.complex128, device=dev)
    stream = torch.cuda.Stream(dev)  # a real (non-null) stream: the library launches on it, events time it
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream

    if not kshard:
        model = _lib.DeviceModel(means, covs, w, device=local)
        if args.precision != "f64":
            model.set_precision(args.precision)
        dm = model

        def step(ev=None):
            model.prepare(None, cfg["snr"], cfg["n_bits"], *qargs, stream=sptr)
            if ev is not None:
                ev[0][0].record(stream)
            model.estimate(yd, _lib.MODE_ALL, 0.0, out=out, stream=sptr)
            if ev is not None:
                ev[0][1].record(stream)
            return None, out
    elif native:
        from quantized_channel_estimation_amd.sharding import make_comm
        comm_kind = args.comm if args.comm != "auto" else ("host" if world > ndev else "rccl")
        comm = make_comm(rank, world, local, kind=comm_kind)
        shard = ComponentShardEstimator(means, covs, w, rank, world, device=local, precision=args.precision,
                                        comm=comm, double_buffer=not args.single_buffer)
        dm = shard.dev

        def step(ev=None):
            # the library's step: prepare + shift MAX, chunked partials + RCCL reduce-scatters, flag MAX; no host sync
            shard.prepare(None, cfg["snr"], cfg["n_bits"], *qargs, stream=sptr)
            return shard.estimate(yd, chunks=args.chunks or None, scatter=args.collective == "rs", sync=False)
    else:
        shard = ComponentShardEstimator(means, covs, w, rank, world, device=local, precision=args.precision)
        dm = shard.dev
        # time only the partial kernels on the compute stream (the collectives run on RCCL's stream)
        orig = shard.dev.partial_shifted

        def step(ev=None):
            shard.prepare(None, cfg["snr"], cfg["n_bits"], *qargs, stream=sptr)
            if ev is not None:
                def timed(*a, **kw):
                    e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    ev.append(e)
                    e[0].record(stream)
                    r = orig(*a, **kw)
                    e[1].record(stream)
                    return r
                shard.dev.partial_shifted = timed
            try:
                # no host sync inside a step: the flag word is read once per timed region (shard.finish)
                return shard.estimate(yd, chunks=args.chunks or None, scatter=args.collective == "rs", sync=False)
            finally:
                shard.dev.partial_shifted = orig

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()

    def finish(res):
        # K-shard: the natural sync point of a run of steps -- Cholesky failures raise, flagged rows are recombined
        return shard.finish() if kshard else res

    res = None
    for _ in range(args.warmup):
        res = step()
    if args.warmup > 0:
        finish(res)
    barrier()
    if kshard and native:
        shard.native.timing(True)  # HIP events around every partial launch on the compute stream (qce_kshard_timing)
        events = None
    elif kshard:
        events = [[] for _ in range(args.steps)]  # filled per chunk by the timed partial launches
    else:
        events = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))]
                  for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        res = step(None if events is None else events[i])
    res = finish(res)
    barrier()
    elapsed = time.perf_counter() - t0
    if events is None:
        tot, _ = shard.native.kernel_ms()
        shard.native.timing(False)
        kern_ms = tot / args.steps
    else:
        kern_ms = float(np.mean([sum(a.elapsed_time(b) for a, b in evs) for evs in events]))
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device="cpu" if native else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    ms_per_step = elapsed / args.steps * 1e3
    total_units = B if kshard else B * world  # K-shard: the node estimates B once; batch: B per rank
    value = total_units * args.steps / elapsed

    # parity + MSE of this rank's last result against the FP64 oracle on a subset
    parity = mse = None
    ho = None
    n_chk = min(B, 512)
    rows, hres = res
    if rank == 0:
        hg = hres.cpu().numpy()
        idx = np.arange(B) if rows is None else rows.cpu().numpy()
        mse = float(np.mean(np.abs(hg - h[idx]) ** 2))
        if not args.no_parity:
            from oracle import qce_oracle as O
            sel = idx[:n_chk]
            ho = O.estimate(means, covs, w, y[sel], cfg["snr"], N, None, "all", cfg["n_bits"], cfg["qtype"],
                            quantizer)
            parity = dict(samples=int(sel.size),
                          rel_fro=float(np.linalg.norm(hg[:n_chk] - ho) / np.linalg.norm(ho)),
                          mse_gpu=float(np.mean(np.abs(hg[:n_chk] - h[sel]) ** 2)),
                          mse_oracle=float(np.mean(np.abs(ho - h[sel]) ** 2)))

    # roofline of the dominant kernel (per rank)
    k_local = (lambda s: s[1] - s[0])(component_slices(K, world)[rank]) if kshard else K
    kern_tag = "fft" if dm.structure()[2] else ("f64" if dtype_of(dm) == "f64" else "h2")
    traffic = None
    tpath = args.traffic or os.path.join(ROOT, "profiles",
                                         f"traffic_{args.config}{'_mean' if args.mean else ''}.json")
    traffic_note = None
    if os.path.exists(tpath):
        try:
            tj = json.load(open(tpath))
            if tj.get("build_id") != _lib.build_id():
                # a PMC measurement of another build of the kernel is not this kernel's traffic
                traffic_note = f"{os.path.basename(tpath)} is from build {tj.get('build_id')}, not {_lib.build_id()}"
            elif tj.get("config") == args.config and tj.get("B") == B and tj.get("kernel") == kern_tag \
                    and not kshard:
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception as e:
            traffic, traffic_note = None, f"unreadable traffic file: {e}"
    roofline = roofline_line(args, cfg, dm, k_local, B, kern_ms, traffic)
    if traffic is not None:
        roofline["traffic_source"] = os.path.relpath(tpath, ROOT) + " (rocprofv3 PMC of this build)"
        if tj.get("dram"):
            roofline["traffic_dram"] = tj["dram"].get("bytes_per_launch")
    elif traffic_note:
        roofline["traffic_note"] = traffic_note

    extras = {}
    if rank == 0 and world == 1 and not args.no_extras and args.config == "metric":
        extras["fast_path"] = fast_line(cfg, means, covs, w, yd, out, stream, max(3, args.steps // 2), qargs, ho,
                                        n_chk)
    if rank == 0 and world == 1 and args.dropin:
        extras["dropin"] = dropin_line(cfg, means, covs, w, y, quantizer)
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "channel estimates/s",
            "n_gpus": world,
            "world_size": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.shard == "k" else "weak",
            "vs_baseline": None,
            "dtype": dtype_of(dm),
            "data": f"synthetic: seeded {cfg['cov']} SCM-derived covariances, SCM channel pool + fresh CN noise, "
                    f"{cfg['n_bits']}-bit {cfg['qtype']} quantised",
            "config": {"workload": f"estimate_from_y K={K} N=M={N} cov={cfg['cov']}{' with means' if args.mean else ''} n_bits={cfg['n_bits']} "
                                   f"{cfg['qtype']} snr={cfg['snr']}dB mode=all B={B}"
                                   f"{'' if args.shard == 'k' else '/GPU'} prepare-per-step",
                       "K": K, "N": N, "B": B, "shard": args.shard,
                       "parallelism": f"{'kshard' if args.shard == 'k' else 'batch'}{world}",
                       "chunks": (args.chunks or default_chunks(world)) if kshard else None,
                       "collectives": (("libqce RCCL communicator (qce_kshard_*)" if comm_kind == "rccl" else
                                        "libqce host transport over gloo (qce_kshard_*; ranks share a GPU)") if native
                                       else f"torch.distributed {args.backend}") if kshard else None},
            "mse": mse,
            "parity": parity,
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        line.update(extras)
        print(json.dumps(line), flush=True)
    # explicit teardown while every rank and the runtimes are still here (not left to exit-time destructors)
    torch.cuda.synchronize(dev)
    if kshard:
        shard.close()
        if native:
            comm.close()
    else:
        model.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
