"""A/B timing of library builds (variant .so files built with `python -m quantized_channel_estimation_amd.build
--variant NAME --define X=Y [--only qce_f64g]`), each timed in its own process, the variants interleaved over
rounds on the same box.  One JSON line per variant: median / min kernel ms of the estimate launch (HIP events,
device-resident y), and ĥ's max relative deviation from the first variant's.
python tools/lib_ab.py --config metric [--rounds 3] main:quantized_channel_estimation_amd/libqce.so e5:...libqce_e5.so"""
import argparse
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(config, launches, out_path, mean=False, components=0):
    sys.path.insert(0, ROOT)
    import torch
    from bench import CONFIGS, make_inputs
    from quantized_channel_estimation_amd import _lib
    cfg = dict(CONFIGS[config])
    if cfg.pop("dense", False):
        os.environ["QCE_FFT"] = "0"
    cfg["mean"] = mean  # as bench.py --mean
    if components:
        cfg["K"] = components  # as bench.py --components (a K-shard rank's share)
    means, covs, w, h, y, qz = make_inputs(cfg, 0)
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    yd = torch.from_numpy(y).to(dev)
    out = torch.empty((cfg["B"], cfg["N"]), dtype=torch.complex128, device=dev)
    m = _lib.DeviceModel(means, covs, w)
    qk = {"uniform": _lib.QUANT_UNIFORM, "lloyd": _lib.QUANT_LLOYD}[cfg["qtype"]]
    thr, lab = (qz[0], qz[1]) if cfg["n_bits"] not in (1, np.inf) and cfg["qtype"] == "lloyd" else (None, None)
    m.prepare(None, cfg["snr"], cfg["n_bits"], qk, thr, lab, stream=st.cuda_stream)
    for _ in range(2):
        m.estimate(yd, out=out, stream=st.cuda_stream)
    torch.cuda.synchronize()
    ts = []
    for _ in range(launches):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        m.estimate(yd, out=out, stream=st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    np.save(out_path, out[:4096].cpu().numpy())
    print(json.dumps({"kernel_ms": ts, "kernel": m.kernel(), "build": _lib.build_id()}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="metric")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--child", default=None)
    ap.add_argument("--mean", action="store_true", help="components with means (as bench.py --mean)")
    ap.add_argument("--components", type=int, default=0, help="K override (as bench.py --components)")
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    if a.child:
        return child(a.config, a.launches, a.child, a.mean, a.components)
    res = {}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    for rnd in range(a.rounds):
        for v in a.variants:
            name, lib = v.split(":", 1)
            env = dict(os.environ, QCE_LIB=os.path.abspath(os.path.join(ROOT, lib)))
            outp = os.path.join(ROOT, "gpurun_out", f"ab_{name}.npy")
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "--config", a.config, "--launches",
                                str(a.launches), "--child", outp] + (["--mean"] if a.mean else []) +
                               (["--components", str(a.components)] if a.components else []), env=env, capture_output=True, text=True,
                               timeout=300)
            if p.returncode != 0:
                print(json.dumps({"variant": name, "error": p.stderr[-2000:]}), flush=True)
                return 1
            r = json.loads(p.stdout.strip().splitlines()[-1])
            res.setdefault(name, {"ms": [], "kernel": r["kernel"], "build": r["build"]})["ms"] += r["kernel_ms"]
    first = None
    for v in a.variants:
        name = v.split(":", 1)[0]
        hv = np.load(os.path.join(ROOT, "gpurun_out", f"ab_{name}.npy"))
        first = hv if first is None else first
        r = res[name]
        print(json.dumps({"variant": name, "config": a.config, "kernel": r["kernel"], "build": r["build"],
                          "median_ms": round(float(np.median(r["ms"])), 4), "min_ms": round(float(np.min(r["ms"])), 4),
                          "h_rel_dev": float(np.abs(hv - first).max() / np.abs(first).max())}), flush=True)


if __name__ == "__main__":
    sys.exit(main())
