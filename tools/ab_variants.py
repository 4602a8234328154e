"""A/B timing of estimate-kernel variants in ONE process (interleaved rounds, MI355X rule 24).
Variants are selected through the library's environment switches (read at every launch)."""
import json, os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bench import CONFIGS, make_inputs
from quantized_channel_estimation_amd import _lib

variants = {
    "deep8": {},
    "wide4": {"QCE_H2_WIDE": "1"},
}
extra = json.loads(sys.argv[1]) if len(sys.argv) > 1 else {}
variants.update(extra)
cfg = dict(CONFIGS["metric"])
means, covs, w, h, y, qz = make_inputs(cfg, 0)
dev = torch.device("cuda", 0)
st = torch.cuda.Stream(dev)
torch.cuda.set_stream(st)
yd = torch.from_numpy(y).to(dev)
out = torch.empty((cfg["B"], cfg["N"]), dtype=torch.complex128, device=dev)
m = _lib.DeviceModel(means, covs, w)
m.prepare(None, cfg["snr"], cfg["n_bits"], stream=st.cuda_stream)
res = {k: [] for k in variants}
ref = None
for rnd in range(6):
    for name, env in variants.items():
        for k in ("QCE_H2_WIDE", "QCE_KERNEL", "QCE_WORKGROUPS"):
            os.environ.pop(k, None)
        os.environ.update(env)
        m.estimate(yd, out=out, stream=st.cuda_stream)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(5):
            m.estimate(yd, out=out, stream=st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        res[name].append(e0.elapsed_time(e1) / 5)
        hv = out.cpu().numpy()
        if ref is None:
            ref = hv
        err = float(np.linalg.norm(hv - ref) / np.linalg.norm(ref))
        if err > 1e-5:
            print("MISMATCH", name, err)
for name, v in res.items():
    print(f"{name:12s} median {np.median(v):.4f} ms  min {np.min(v):.4f} ms  -> {cfg['B']/np.median(v)*1e3/1e6:.1f} M est/s")
