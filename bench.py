#!/usr/bin/env python3
"""Throughput of the MI355X Bussgang-GMM estimate path (BASELINE.json metric).

A step is one ``estimate_from_y`` of the reference (gmm_cplx_bussgang.py:166-243) over one batch:
the per-SNR FP64 precompute (prepare) followed by the fused estimate kernel, with the batch of
quantised observations already resident in HBM.  Default workload = the metric configuration
(SURVEY.md §8(d) D2): K=128 components, N=M=64 antennas, 'full' covariances, 1-bit uniform
quantiser, SNR 5 dB, mode 'all', B=100,000 observations per GPU.

  python bench.py [--gpus N --steps K --warmup W] [--config metric|cfg1..cfg5|cfg3dense|cfg5dense]
                  [--shard batch|k]

cfg3 / cfg5 are (block-)circulant mixtures with A = I: they take the Fourier-domain path
(qce_fft.hip, HBM-bound roofline); the *dense variants force the dense path (QCE_FFT=0).

Multi-GPU (launched by torch.distributed.run, one rank per GPU): ``--shard batch`` (default) gives
every rank its own B observations and the whole mixture (no data-path collective, weak scaling);
``--shard k`` splits the K components over the ranks and combines with one RCCL all-reduce
(strong scaling).  Rank 0 prints one JSON line.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "channel estimates/sec + MSE vs reference; K=128 N=64 full-cov, 1/2/4/8 GPU"
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak (spec)
FP64_MFMA_PEAK_TFLOPS = 78.6  # MI355X_MICROARCH.md / SURVEY D3: v_mfma_f64_16x16x4_f64 dense peak (spec)
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="metric", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0, help="override B (observations per GPU)")
    ap.add_argument("--shard", default="batch", choices=["batch", "k"])
    ap.add_argument("--precision", default="f64", choices=["f64", "fast"],
                    help="dense 'all' arithmetic: f64 (reference complex128, default) or fast (fp16 split)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline budget (0 = skip)")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic_metric.json"),
                    help="JSON with PMC-derived HBM bytes per launch of the estimate kernel")
    return ap.parse_args()


def make_inputs(cfg, seed, pool=2048):
    """Synthetic batch of the configured shape: SCM channels (a seeded pool of `pool` distinct
    channels, reused with fresh noise) -> quantised observations y = Q(h + n)."""
    from quantized_channel_estimation_amd import inputs
    K, N, B = cfg["K"], cfg["N"], cfg["B"]
    means, covs, w = inputs.synthetic_model(K, N, cov_type=cfg["cov"], blocks=cfg.get("blocks"))
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


def cpu_baseline(cfg, means, covs, w, y, quantizer, budget_s):
    """Loop-faithful oracle (the reference's per-(sample, component) op order) on a bounded
    sample of the same workload, single thread."""
    from oracle import qce_oracle as O
    try:
        from threadpoolctl import threadpool_limits
        lim = threadpool_limits(limits=1)
    except Exception:  # pragma: no cover
        lim = None
    N = cfg["N"]
    def run(n):
        t0 = time.perf_counter()
        O.estimate_loop(means, covs, w, y[:n], cfg["snr"], N, None, cfg["n_bits"], cfg["qtype"], quantizer)
        return time.perf_counter() - t0
    a, b = (4, 36) if N <= 64 else (1, 3)  # N >= 128: one loop-faithful estimate costs ~0.1-2 s
    t1, t2 = run(a), run(b)
    per = max((t2 - t1) / (b - a), 1e-6)
    prep = max(t1 - a * per, 0.0)
    n = int(max(b, min(y.shape[0], (budget_s - prep) / per)))
    t0 = time.perf_counter()
    O.estimate_loop(means, covs, w, y[:n], cfg["snr"], N, None, cfg["n_bits"], cfg["qtype"], quantizer)
    dt = time.perf_counter() - t0
    if lim is not None:
        lim.unregister()
    return dict(value=n / dt, unit="estimates/s", cores=1, kind="port",
                sample=f"{n} observations of the same workload through oracle.estimate_loop (per-call prepare "
                       f"included, 1 BLAS thread), {dt:.1f} s")


def main():
    args = parse()
    cfg = dict(CONFIGS[args.config])
    if cfg.pop("dense", False):
        os.environ["QCE_FFT"] = "0"  # read by qce_prepare: keep the structured mixture on the dense path
    import torch
    import torch.distributed as dist
    from quantized_channel_estimation_amd import _lib
    from quantized_channel_estimation_amd.sharding import ComponentShardEstimator, component_slices

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if args.batch:
        cfg["B"] = args.batch
    K, N, B = cfg["K"], cfg["N"], cfg["B"]
    data_seed = rank if args.shard == "batch" else 0
    means, covs, w, h, y, quantizer = make_inputs(cfg, data_seed)
    qkind = {"uniform": _lib.QUANT_UNIFORM, "lloyd": _lib.QUANT_LLOYD}[cfg["qtype"]]
    thr, lab = (quantizer[0], quantizer[1]) if cfg["n_bits"] not in (1, np.inf) and cfg["qtype"] == "lloyd" else \
        (None, None)

    dev = torch.device("cuda", local)
    yd = torch.from_numpy(y).to(dev)
    out = torch.empty((B, N), dtype=torch.complex128, device=dev)
    stream = torch.cuda.Stream(dev)  # a real (non-null) stream: the library launches on it, events time it
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream

    if args.shard == "batch":
        model = _lib.DeviceModel(means, covs, w, device=local)
        if args.precision != "f64":
            model.set_precision(args.precision)

        def step(ev=None):
            model.prepare(None, cfg["snr"], cfg["n_bits"], qkind, thr, lab, stream=sptr)
            if ev is not None:
                ev[0].record(stream)
            model.estimate(yd, _lib.MODE_ALL, 0.0, out=out, stream=sptr)
            if ev is not None:
                ev[1].record(stream)
            return out
    else:
        shard = ComponentShardEstimator(means, covs, w, rank, world, device=local)
        m_b = torch.empty(B, dtype=torch.float64, device=dev)
        s_b = torch.empty(B, dtype=torch.float64, device=dev)
        a_b = torch.empty((B, 2 * N), dtype=torch.float32, device=dev)
        from quantized_channel_estimation_amd.sharding import combine_partials_dist

        def step(ev=None):
            shard.prepare(None, cfg["snr"], cfg["n_bits"], qkind, thr, lab, stream=sptr)
            if ev is not None:
                ev[0].record(stream)
            shard.dev.partial(yd, m_b, s_b, a_b, stream=sptr)
            if ev is not None:
                ev[1].record(stream)
            return combine_partials_dist(m_b, s_b, a_b, shard.shift, N)

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    barrier()
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        res = step(events[i])
    barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in events]))
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    ms_per_step = elapsed / args.steps * 1e3
    total_units = B * world if args.shard == "batch" else B
    value = total_units * args.steps / elapsed

    # parity + MSE of this rank's last result against the FP64 oracle on a subset
    parity = None
    mse = None
    if rank == 0:
        hg = res.cpu().numpy()
        mse = float(np.mean(np.abs(hg - h) ** 2))
        if not args.no_parity:
            from oracle import qce_oracle as O
            n_chk = min(B, 512)
            ho = O.estimate(means, covs, w, y[:n_chk], cfg["snr"], N, None, "all", cfg["n_bits"], cfg["qtype"],
                            quantizer)
            parity = dict(samples=n_chk,
                          rel_fro=float(np.linalg.norm(hg[:n_chk] - ho) / np.linalg.norm(ho)),
                          mse_gpu=float(np.mean(np.abs(hg[:n_chk] - h[:n_chk]) ** 2)),
                          mse_oracle=float(np.mean(np.abs(ho - h[:n_chk]) ** 2)))

    # roofline of the dominant kernel
    k_local = K if args.shard == "batch" else (lambda s: s[1] - s[0])(component_slices(K, world)[rank])
    dm = model if args.shard == "batch" else shard.dev
    fourier = bool(dm.structure()[2])
    f32_kernel = os.environ.get("QCE_KERNEL") == "f32"
    traffic = None
    kern_tag = "fft" if fourier else ("f32" if f32_kernel else "h2")
    if os.path.exists(args.traffic):
        try:
            tj = json.load(open(args.traffic))
            if tj.get("config") == args.config and tj.get("B") == B and tj.get("kernel") == kern_tag:
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    if fourier:
        # HBM-bound: 16 M bytes of y in + 16 N bytes of h out per estimate (c128)
        bytes_per_launch = 32.0 * N * B
        achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
        n1, n2, _ = dm.structure()
        fft_flops = (4.0 * k_local * N + 10.0 * N * math.log2(N)) * B  # D3: zero-mean FFT-path flops
        roofline = dict(bound="hbm", achieved=round(achieved, 2), peak=HBM_PEAK_GBS, unit="GB/s",
                        frac=round(achieved / HBM_PEAK_GBS, 4), traffic=traffic,
                        kernel="k_fft_est", structure=f"block-circulant ({n1},{n2})" if n1 > 1 else "circulant",
                        kernel_ms=round(kern_ms, 4), bytes_per_launch=bytes_per_launch,
                        fp64_flops_per_launch=fft_flops,
                        fp64_tflops=round(fft_flops / (kern_ms * 1e-3) / 1e12, 3))
    else:
        flops_per_launch = 16.0 * k_local * N * N * B  # 16 K M N real flops / estimate
        achieved = flops_per_launch / (kern_ms * 1e-3) / 1e12
        if args.precision == "f64" and not f32_kernel and N <= 64:
            # FP64 kernel: executed v_mfma_f64_16x16x4 work = 256 flops per sample per 1 KB table block
            # (GL: NTL(NTL+1) blocks, Linv's upper triangle skipped; GW: NTW * KP blocks)
            Np = 16 if N <= 16 else (32 if N <= 32 else 64)
            ntl, ntw, kp = Np // 8, Np // 8, Np // 4
            executed = 256.0 * (ntl * (ntl + 1) + ntw * kp) * k_local * B
            roofline = dict(bound="mfma", achieved=round(achieved, 3), peak=FP64_MFMA_PEAK_TFLOPS, unit="TFLOP/s",
                            frac=round(achieved / FP64_MFMA_PEAK_TFLOPS, 4), traffic=traffic,
                            kernel="k_est_all_f64 (+k_merge_f64)", peak_dtype="fp64 MFMA (dense)",
                            kernel_ms=round(kern_ms, 4), flops_per_launch=flops_per_launch,
                            executed_flops_per_launch=executed,
                            mfma_issue_frac=round(executed / (kern_ms * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS, 4))
        peak = FP32_MFMA_PEAK_TFLOPS if f32_kernel else FP16_MFMA_PEAK_TFLOPS
        # executed MFMA work: lower-triangular tiles of E(Linv) skipped (R/32 slices of 32x16 tiles) and,
        # for the fp16 kernel, two products (hi, lo) per fp32-class MAC
        nsl = (2 * N) // 32
        tri = (sum(2 * r + 2 for r in range(nsl)) / (nsl * 2 * nsl) + 1.0) / 2.0
        executed = flops_per_launch * tri * (1.0 if f32_kernel else 2.0)
        if not (args.precision == "f64" and not f32_kernel and N <= 64):
          roofline = dict(bound="mfma", achieved=round(achieved, 3), peak=peak, unit="TFLOP/s",
                        frac=round(achieved / peak, 4), traffic=traffic,
                        kernel=("k_est_all_f32" if f32_kernel else "k_est_all_h2+k_merge_streamk"),
                        peak_dtype="fp32 MFMA" if f32_kernel else "fp16 MFMA (dense)",
                        kernel_ms=round(kern_ms, 4), flops_per_launch=flops_per_launch,
                        mfma_issue_frac=round(executed / (kern_ms * 1e-3) / 1e12 / peak, 4))

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(cfg, means, covs, w, y, quantizer, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "channel estimates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak" if args.shard == "batch" else "strong",
            "vs_baseline": None,
            "dtype": "f64" if (fourier or (args.precision == "f64" and not f32_kernel and N <= 64)) else (
                "f32" if f32_kernel else "f16x2 (fp16 hi+lo split, fp32 accumulate, fp64 softmax)"),
            "data": f"synthetic: seeded {cfg['cov']} SCM-derived covariances, SCM channel pool + fresh CN noise, "
                    f"{cfg['n_bits']}-bit {cfg['qtype']} quantised",
            "config": {"workload": f"estimate_from_y K={K} N=M={N} cov={cfg['cov']} n_bits={cfg['n_bits']} "
                                   f"{cfg['qtype']} snr={cfg['snr']}dB mode=all B={B}/GPU prepare-per-step",
                       "K": K, "N": N, "B_per_gpu": B, "shard": args.shard,
                       "parallelism": f"{args.shard}{world}"},
            "mse": mse,
            "parity": parity,
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
