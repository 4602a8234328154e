"""One rank's share of the N-GPU K-shard step on one GPU (N = 8, 4, 2: K/N of the metric config's 128 components),
the whole batch B = 1e5, the shifted packed partial (qce_estimate_partial_shifted) in 1, 2, 4 or 8 chunks -- the
kernel work a rank does per step besides its reduce-scatters.  Prints the per-step time (HIP events around the
prepare and the chunk loop)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from quantized_channel_estimation_amd import _lib
    cfg = dict(bench.CONFIGS["metric"])
    means, covs, w, h, y, qz = bench.make_inputs(cfg, 0)
    K, N, B = cfg["K"], cfg["N"], cfg["B"]
    yd = torch.from_numpy(y).to("cuda")
    st = torch.cuda.current_stream().cuda_stream
    out = torch.empty((B, 2 * N + 2), dtype=torch.float64, device="cuda")
    for ranks, chunks in [(r, c) for r in (8, 4, 2) for c in (1, 2, 4, 8)]:
        lo, hi = 0, K // ranks
        dm = _lib.DeviceModel(means[lo:hi], covs[lo:hi], w[lo:hi])
        dm.prepare(None, cfg["snr"], float(cfg["n_bits"]), stream=st)
        shift = torch.tensor([max(float(x) for x in dm.cconst())], dtype=torch.float64, device="cuda")
        step = -(-B // chunks)

        def run():
            dm.prepare(None, cfg["snr"], float(cfg["n_bits"]), stream=st)
            for c in range(chunks):
                a, b = c * step, min(B, (c + 1) * step)
                dm.partial_shifted(yd[a:b], shift, out=out[a:b], stream=st)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(f"ranks {ranks} chunks {chunks}: {ms:.4f} ms per step (prepare + {chunks} partial launches over B={B}, "
              f"K_local={hi - lo})", flush=True)
        dm.close()


if __name__ == "__main__":
    main()
