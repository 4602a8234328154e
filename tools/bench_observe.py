"""Throughput of the on-device observation kernel (qce_observe: y = Q(h + s w), csrc/qce_observe.hip)
against the HBM roofline.  Algorithmic bytes per complex element: 16 (h) + 16 (y), + 16 when the
noise w is supplied.  Inputs resident in HBM; HIP events on torch's current stream (the stream the
kernel is launched on).  Prints one JSON line per variant."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantized_channel_estimation_amd import inputs, observe  # noqa: E402

HBM_PEAK = 8000.0  # GB/s, MI355X_MICROARCH.md


def run(name, fn, n_elem, bytes_per_elem, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    gbs = n_elem * bytes_per_elem / (ms * 1e-3) / 1e9
    print(json.dumps({"kernel": "k_observe_id", "variant": name, "elements": n_elem, "ms": round(ms, 4),
                      "achieved_GBs": round(gbs, 1), "peak_GBs": HBM_PEAK, "frac": round(gbs / HBM_PEAK, 4),
                      "observations_per_s": round(n_elem / 64 / (ms * 1e-3), 1)}), flush=True)


def main():
    B, N = int(os.environ.get("OBS_B", 1_000_000)), 64
    g = torch.Generator(device="cuda").manual_seed(0)
    h = torch.randn((B, N), dtype=torch.complex128, device="cuda", generator=g)
    w = torch.randn((B, N), dtype=torch.complex128, device="cuda", generator=g)
    thr, lab, _ = inputs.get_quantizer([5.0], 3, "lloyd")[5.0]
    n = B * N
    run("1bit_generated_noise", lambda: observe.get_observation_nbit(h, 5.0, None, 1, seed=1), n, 32)
    run("3bit_lloyd_generated_noise", lambda: observe.get_observation_nbit(h, 5.0, None, 3, thr, lab, seed=1), n, 32)
    run("1bit_supplied_noise", lambda: observe.get_observation_nbit(h, 5.0, None, 1, noise=w), n, 48)
    run("inf_generated_noise", lambda: observe.get_observation_nbit(h, 5.0, None, np.inf, seed=1), n, 32)
    run("sq_error", lambda: observe.sq_error(h, w), n, 32)


if __name__ == "__main__":
    main()
