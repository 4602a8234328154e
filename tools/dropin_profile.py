"""Drop-in numpy path: per-call time of DeviceModel.estimate / Gmm_nbit.estimate_from_y with
numpy y in and numpy h out at the metric configuration, against the device-resident call, over the direct-DMA
pipeline's chunk plans (QCE_HOST_C0 first-chunk rows, QCE_HOST_GROW growth).  One JSON line per variant.
python tools/dropin_profile.py"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch
    from quantized_channel_estimation_amd import Gmm_nbit, _lib
    cfg = dict(bench.CONFIGS["metric"])
    means, covs, w, h, y, quantizer = bench.make_inputs(cfg, 0)
    dm = _lib.DeviceModel(means, covs, w)
    yd = torch.from_numpy(y).cuda()

    def timeit(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        return float(np.median(ts)), float(np.min(ts))

    def dev_call():
        dm.prepare(None, cfg["snr"], 1)
        dm.estimate(yd)
    print(json.dumps({"variant": "device-resident prepare+estimate", "ms": timeit(dev_call)}), flush=True)
    ref = None
    for c0, grow in [(None, None), (2048, 4), (8192, 4), (16384, 2), (32768, 2), (4096, 8), (12500, 1),
                     (25000, 1), (50000, 1)]:
        for k, v in (("QCE_HOST_C0", c0), ("QCE_HOST_GROW", grow)):
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = str(v)

        def host_call():
            dm.prepare(None, cfg["snr"], 1)
            return dm.estimate(y)
        hr = host_call()
        ref = hr.copy() if ref is None else ref
        print(json.dumps({"variant": f"host numpy c0={c0} grow={grow}", "ms": timeit(host_call),
                          "max_rel_diff": float(np.abs(hr - ref).max() / np.abs(ref).max())}), flush=True)
    os.environ.pop("QCE_HOST_C0", None)
    os.environ.pop("QCE_HOST_GROW", None)
    os.environ["QCE_HOST_DIRECT"] = "0"
    print(json.dumps({"variant": "staged pipeline (round 4)", "ms": timeit(lambda: (dm.prepare(None, cfg['snr'], 1),
                                                                                     dm.estimate(y)))}), flush=True)
    os.environ.pop("QCE_HOST_DIRECT")
    g = Gmm_nbit.from_params(means, covs, w)
    args = (cfg["snr"], cfg["N"], None, "all", 1, cfg["qtype"], quantizer)
    print(json.dumps({"variant": "Gmm_nbit.estimate_from_y", "ms": timeit(lambda: g.estimate_from_y(y, *args))}),
          flush=True)
    t0 = time.perf_counter()
    yc = np.ascontiguousarray(y, dtype=np.complex128)
    print(json.dumps({"variant": "python ascontiguousarray(y)", "ms": (time.perf_counter() - t0) * 1e3}), flush=True)


if __name__ == "__main__":
    main()
