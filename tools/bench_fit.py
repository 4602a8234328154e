"""One device EM iteration at the training scale of the reference scripts (K=128 components,
N=64 antennas, B=100k channels) against the FP64 MFMA roofline, next to the
oracle's NumPy E/M-steps (the reference's arithmetic) on a bounded sample of the same data.

M-step algorithmic flops: 8 K B N^2 (the K weighted Hermitian covariance products; complex MAC = 8).
E-step algorithmic flops: 8 K B N^2 (K triangular whitenings counted as full M x M products, the
SURVEY D3 convention for the log-prob).  Times are HIP events on torch's current stream (the one
the library launches on).  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantized_channel_estimation_amd import _em, inputs  # noqa: E402

FP64_PEAK = 78.6  # TFLOP/s, MI355X FP64 matrix (spec)


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    K, N, B = 128, 64, int(os.environ.get("FIT_B", 100_000))
    means, covs, w = inputs.synthetic_model(K, N)
    rng = np.random.default_rng(5)
    hp, _ = inputs.scm_generate(4096, 1, N, rng, n_path=3)
    X = hp[rng.integers(0, 4096, size=B), 0, :].astype(np.complex128)
    X = X + 0.05 * (rng.standard_normal(X.shape) + 1j * rng.standard_normal(X.shape))
    em = _em.DeviceEM(X, K, "full", 1e-6, True)
    R0 = rng.random((B, K))
    R0 /= R0.sum(axis=1, keepdims=True)
    em.R.copy_(torch.from_numpy(R0))
    flops = 8.0 * K * B * N * N
    ms_m = timed(lambda: em.mstep(), 5)
    ms_e = timed(lambda: em.estep(means, covs, w), 5)
    out = {"workload": f"EM iteration K={K} N={N} B={B} full, zero-mean", "mstep_ms": round(ms_m, 3),
           "estep_ms": round(ms_e, 3), "iteration_ms": round(ms_m + ms_e, 3),
           "mstep_tflops": round(flops / (ms_m * 1e-3) / 1e12, 2), "estep_tflops": round(flops / (ms_e * 1e-3) / 1e12, 2),
           "fp64_peak_tflops": FP64_PEAK, "mstep_frac": round(flops / (ms_m * 1e-3) / 1e12 / FP64_PEAK, 4),
           "note": "mstep/estep times include host copies of the K x N x N parameters and the device model build"}
    cpu_s = float(os.environ.get("FIT_CPU_SECONDS", 10))
    if cpu_s > 0:
        from oracle import qce_oracle as O
        try:
            from threadpoolctl import threadpool_limits
            lim = threadpool_limits(limits=1)
        except Exception:
            lim = None
        Bs = 2000
        Xs, Rs = X[:Bs], R0[:Bs]
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < cpu_s:
            O.em_mstep(Xs, Rs, 1e-6, "full", True)
            P = O.precision_cholesky(covs)
            O.log_prob_resp(Xs, means, P, w)
            n += 1
        dt = (time.perf_counter() - t0) / n
        out["cpu_baseline"] = {"iteration_s_at_B": round(dt * B / Bs, 3), "cores": 1, "kind": "port",
                               "sample": f"{n} oracle E+M iterations on {Bs} of the {B} channels, scaled linearly"}
        out["speedup_vs_cpu_1core"] = round(dt * B / Bs / ((ms_m + ms_e) * 1e-3), 1)
        del lim
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
