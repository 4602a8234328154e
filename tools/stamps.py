"""Run the metric workload on the QCE_STAMPS diagnostic library and print per-segment cycle shares
of the deep loop (GL, softmax, barrier0, GWa, barrier1, GWb, barrier2)."""
import ctypes, os, sys
import numpy as np
os.environ["QCE_LIB"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                      "quantized_channel_estimation_amd", "libqce_stamps.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bench import CONFIGS, make_inputs
from quantized_channel_estimation_amd import _lib
cfg = dict(CONFIGS["metric"])
means, covs, w, h, y, qz = make_inputs(cfg, 0)
y = torch.from_numpy(y).cuda()
m = _lib.DeviceModel(means, covs, w)
m.prepare(None, cfg["snr"], cfg["n_bits"])
lib = _lib.load()
for _ in range(2):
    m.estimate(y)
buf = np.zeros(4096 * 64, dtype=np.uint64)
f = lib.qce_debug_stamps
f.argtypes = [ctypes.c_void_p, ctypes.c_int]
f.restype = ctypes.c_int
assert f(buf.ctypes.data, buf.size) == 0
a = buf.reshape(4096, 8, 8)[:, :, :7].astype(np.float64)
tot = a.sum(axis=(0, 1))
names = ["GL", "softmax", "bar0", "GWa", "bar1", "GWb", "bar2"]
print("share:", {n: round(float(v / tot.sum()), 3) for n, v in zip(names, tot)})
per_wave = a.sum(axis=2)
nz = per_wave[per_wave > 0]
print("waves with stamps", nz.size, "mean cycles per wave", nz.mean())
# per component: items per workgroup
