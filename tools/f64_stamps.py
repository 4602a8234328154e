"""Segment cycle breakdown of k_est_all_f64 at a bench configuration (default metric; argv[1]: cfg4, ...; argv[2]: K),
diagnostic build.

  python -m quantized_channel_estimation_amd.build --stamps      # libqce_stamps.so
  QCE_LIB=quantized_channel_estimation_amd/libqce_stamps.so python tools/f64_stamps.py
Segments (per wave, s_memtime): 0 GL blocks, 1 softmax, 2 GW blocks, 3 boundary wait (vmcnt + barrier),
4 ring refill issue, 5 tile overhead (y load, drain, write)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from quantized_channel_estimation_amd import _lib
    import bench
    cfg = dict(bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "metric"])
    if len(sys.argv) > 2:  # argv[2]: components (a K-shard rank's share, e.g. 16 of the metric's 128)
        cfg["K"] = int(sys.argv[2])
    means, covs, w, h, y, qz = bench.make_inputs(cfg, 0)
    dm = _lib.DeviceModel(means, covs, w)
    dm.prepare(None, cfg["snr"], 1.0)
    yd = torch.from_numpy(y).to("cuda")
    for _ in range(3):
        dm.estimate(yd)
    dm.synchronize()
    lib = _lib.load()
    fn = lib.qce_debug_f64_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    buf = np.zeros(4096 * 8 * 8, dtype=np.uint64)
    n = fn(buf.ctypes.data, buf.size)
    st = buf[:n].reshape(-1, 8).astype(np.float64)
    st = st[st.sum(1) > 0]
    tot = st.sum(1, keepdims=True)
    names = ["GL", "softmax", "GW", "bnd-wait", "refill", "tile-ovh", "-", "-"]
    frac = (st / tot).mean(0)
    print(f"waves {st.shape[0]}, mean cycles/wave {tot.mean():.4g}")
    for i in range(6):
        print(f"  {names[i]:9s} {frac[i]:.4f}   (max over waves {(st[:, i] / tot[:, 0]).max():.4f})")


if __name__ == "__main__":
    main()
