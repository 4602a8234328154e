"""Host-memory probe for the drop-in numpy path: cost of hipHostRegister / Unregister on touched
and untouched numpy buffers of the metric's size (102.4 MB), and H2D / D2H rates from pageable, registered and
hipHostMalloc'ed memory.  python tools/probe/hostreg_probe.py"""
import ctypes
import json
import time

import numpy as np
import torch

hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipDeviceSynchronize.argtypes = []
H2D, D2H = 1, 2
NB = 100_000 * 64 * 16
dev = torch.empty(NB, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
out = {}


def t(fn, reps=3):
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        best = min(best, time.perf_counter() - t0)
    return best * 1e3


def copy(host, kind):
    def f():
        if kind == H2D:
            assert hip.hipMemcpy(dev.data_ptr(), host, NB, H2D) == 0
        else:
            assert hip.hipMemcpy(host, dev.data_ptr(), NB, D2H) == 0
    return f


a = np.ones(NB, dtype=np.uint8)
out["pageable_h2d_ms"] = t(copy(a.ctypes.data, H2D))
out["pageable_d2h_ms"] = t(copy(a.ctypes.data, D2H))
for touched in (True, False):
    regs, unregs, h2d, d2h = [], [], [], []
    for _ in range(3):
        b = np.ones(NB, dtype=np.uint8) if touched else np.empty(NB, dtype=np.uint8)
        t0 = time.perf_counter()
        assert hip.hipHostRegister(b.ctypes.data, NB, 0) == 0
        regs.append((time.perf_counter() - t0) * 1e3)
        h2d.append(t(copy(b.ctypes.data, H2D), 1))
        d2h.append(t(copy(b.ctypes.data, D2H), 1))
        t0 = time.perf_counter()
        assert hip.hipHostUnregister(b.ctypes.data) == 0
        unregs.append((time.perf_counter() - t0) * 1e3)
        del b
    tag = "touched" if touched else "untouched"
    out[f"register_{tag}_ms"] = regs
    out[f"unregister_{tag}_ms"] = unregs
    out[f"registered_{tag}_h2d_ms"] = h2d
    out[f"registered_{tag}_d2h_ms"] = d2h
p = ctypes.c_void_p()
assert hip.hipHostMalloc(ctypes.byref(p), NB, 0) == 0
out["pinned_h2d_ms"] = t(copy(p.value, H2D))
out["pinned_d2h_ms"] = t(copy(p.value, D2H))
t0 = time.perf_counter()
c = np.empty(NB, dtype=np.uint8)
c[:] = 1
out["numpy_alloc_touch_ms"] = (time.perf_counter() - t0) * 1e3
t0 = time.perf_counter()
np.copyto(c, a)
out["numpy_copy_touched_ms"] = (time.perf_counter() - t0) * 1e3
out["bytes"] = NB
print(json.dumps(out))
