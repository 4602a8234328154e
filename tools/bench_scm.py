"""Throughput of the on-device SCM channel generator (qce_scm_generate, device draws) at the scripts'
training size (N=64 antennas, 100k channels, n_path 3), next to the host restatement of the
reference (inputs.scm_generate, NumPy, 1 thread) on a bounded sample.  FP64 VALU-bound: per channel
and column ~14 F N flops (F = 100 N) for the two partial DFTs.  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantized_channel_estimation_amd import inputs  # noqa: E402
from quantized_channel_estimation_amd.scm import SCMMulti  # noqa: E402


def main():
    B, N = int(os.environ.get("SCM_B", 100_000)), 64
    gen = SCMMulti(2.0, 3)
    gen.generate_channel(1000, 1, N, seed=1, out="device")
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    gen.generate_channel(B, 1, N, seed=2, out="device")
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    F = 100 * N
    flops = 14.0 * F * N * B
    from threadpoolctl import threadpool_limits
    with threadpool_limits(limits=1):
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < 5.0:
            inputs.scm_generate(50, 1, N, np.random.default_rng(n), n_path=3)
            n += 50
        cpu = n / (time.perf_counter() - t0)
    print(json.dumps({"kernel": "k_scm<64>", "channels": B, "N": N, "ms": round(ms, 3),
                      "channels_per_s": round(B / (ms * 1e-3), 1), "fp64_tflops": round(flops / (ms * 1e-3) / 1e12, 2),
                      "cpu_baseline": {"channels_per_s": round(cpu, 1), "cores": 1, "kind": "port",
                                       "sample": f"{n} channels through inputs.scm_generate"},
                      "speedup": round(B / (ms * 1e-3) / cpu, 1)}), flush=True)


if __name__ == "__main__":
    main()
