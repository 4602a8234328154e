"""Segment cycle breakdown of k_fft_wave at cfg3 (or the config named by argv[1]) -- diagnostic build.

  python -m quantized_channel_estimation_amd.build --stamps      # libqce_stamps.so
  QCE_LIB=quantized_channel_estimation_amd/libqce_stamps.so python tools/fft_stamps.py [cfg3]
Segments (per wave, s_memtime, summed over the wave's tiles): 0 y load + LDS write, 1 forward FFT,
2 |Y|^2 + first lp block, 3 component loop, 4 last block + Z, 5 inverse FFT, 6 store."""
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
    cfg = dict(bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "cfg3"])
    means, covs, w, h, y, qz = bench.make_inputs(cfg, 0)
    dm = _lib.DeviceModel(means, covs, w)
    kind = _lib.QUANT_LLOYD if cfg.get("qtype") == "lloyd" else _lib.QUANT_UNIFORM
    dm.prepare(None, cfg["snr"], float(cfg["n_bits"]), kind, qz[0], qz[1])
    yd = torch.from_numpy(y).to("cuda")
    for _ in range(3):
        dm.estimate(yd)
    dm.synchronize()
    lib = _lib.load()
    fn = lib.qce_debug_fft_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    nw = 4096 * 4
    buf = np.zeros(nw * 8, dtype=np.uint64)
    assert fn(buf.ctypes.data, buf.size) == 0  # allocate + enable
    dm.estimate(yd)
    dm.synchronize()
    n = fn(buf.ctypes.data, buf.size)
    fn(None, 0)
    st = buf[:n].reshape(-1, 8).astype(np.float64)
    st = st[st.sum(1) > 0]
    tot = st.sum(1)
    new = os.environ.get("QCE_FFT_CHUNK", "1") != "0"
    if cfg["N"] >= 128 and new:  # k_fft_chunk (zero-mean N = 128, 256)
        names = ["y load", "FFT fwd", "Y regs+|Y|^2", "lp MFMA", "max/e/sums", "filter", "Z+IFFT", "store"]
    elif cfg["N"] == 64 and new:  # k_fft_wreg
        names = ["pass1+xchg", "pass2+stash", "lp0", "loop", "last+Z", "IFFT+store", "sync", "-"]
    else:  # k_fft_wave; k_fft_mfma: 2 = Y regs + lp0, 3 = loop, 4 = Z
        names = ["y load", "FFT fwd", "y2+lp0", "loop", "last+Z", "FFT inv", "store", "-"]
    print(f"waves {st.shape[0]}, mean cycles/wave {tot.mean():.4g} (min {tot.min():.4g}, max {tot.max():.4g})")
    for i in range(8):
        print(f"  {names[i]:8s} {st[:, i].mean() / tot.mean():.4f}  mean {st[:, i].mean():.4g} cycles/wave")


if __name__ == "__main__":
    main()
