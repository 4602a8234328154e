"""Per-SNR prepare time (qce_prepare on its stream, HIP events, median of 20) at a bench configuration; one JSON
line.  Kernel variants through the library's environment switches (QCE_CHOL, QCE_CHOL_THREADS, ...), one
process per variant.  python tools/prepare_time.py [config]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    from quantized_channel_estimation_amd import _lib
    name = sys.argv[1] if len(sys.argv) > 1 else "metric"
    cfg = dict(bench.CONFIGS[name])
    means, covs, w, h, y, qz = bench.make_inputs(dict(cfg, B=256), 0)
    dm = _lib.DeviceModel(means, covs, w)
    st = torch.cuda.Stream()
    for _ in range(3):
        dm.prepare(None, cfg["snr"], cfg["n_bits"], stream=st.cuda_stream)
    torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        dm.prepare(None, cfg["snr"], cfg["n_bits"], stream=st.cuda_stream)
        b.record(st)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    yd = torch.from_numpy(y).cuda()
    hv = dm.estimate(yd).cpu().numpy()
    print(json.dumps({"config": name, "K": cfg["K"], "N": cfg["N"], "prepare_ms_median": float(np.median(ts)),
                      "prepare_ms_min": float(np.min(ts)), "env": {k: v for k, v in os.environ.items()
                                                                   if k.startswith("QCE_CHOL")},
                      "h_checksum": float(np.abs(hv).sum())}), flush=True)


if __name__ == "__main__":
    main()
