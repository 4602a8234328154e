"""One-column vs two-column-per-phase Cholesky (QCE_CHOL_PAIRS) on the same models: the prepared tables
(P = Linv^H, cconst, W, b) must be bit-identical, and the prepare time of each (HIP events, median of 20).  Each variant in its
own process (the switch is read once per process).  python tools/chol_pairs_check.py [--env QCE_CHOL_V3]: any
on/off switch of the factorisation (variant "1" vs "0"; the tables then agree to rounding, max_rel_dev)."""
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [("metric", 128, 64), ("cfg2", 64, 64), ("k16", 16, 64), ("cfg1", 16, 32), ("odd33", 24, 33), ("n63", 8, 63),
         ("odd17", 5, 17), ("odd7", 9, 7), ("one", 3, 1)]


def child(out):
    sys.path.insert(0, ROOT)
    import torch
    from quantized_channel_estimation_amd import _lib, inputs
    res = {}
    for name, K, N in CASES:
        means, covs, w = inputs.synthetic_model(K, N, cov_type="full")
        dm = _lib.DeviceModel(means, covs, w)
        st = torch.cuda.Stream()
        for _ in range(3):
            dm.prepare(None, 5.0, 1, stream=st.cuda_stream)
        torch.cuda.synchronize()
        ts = []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            dm.prepare(None, 5.0, 1, stream=st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        t = dm.tables(["means_y", "Cy", "Cr", "P", "A_eff", "W", "b", "cconst"])
        np.savez(out + f"_{name}.npz", **{k: np.asarray(v) for k, v in t.items()})
        res[name] = float(np.median(ts))
        dm.close()
    print(json.dumps(res))


def main():
    if len(sys.argv) > 1 and sys.argv[1] != "--env":
        return child(sys.argv[1])
    env_name = sys.argv[2] if len(sys.argv) > 2 else "QCE_CHOL_PAIRS"
    scratch = tempfile.mkdtemp(prefix="qce_chol_check_")  # the table dumps (tens of MB) stay off gpurun_out
    times = {}
    for var in ("1", "0"):
        out = os.path.join(scratch, f"chol_pairs{var}")
        p = subprocess.run([sys.executable, os.path.abspath(__file__), out], env=dict(os.environ, **{env_name: var}),
                           capture_output=True, text=True, timeout=300)
        if p.returncode:
            print(p.stderr[-3000:])
            return 1
        times[var] = json.loads(p.stdout.strip().splitlines()[-1])
    for name, K, N in CASES:
        a = np.load(os.path.join(scratch, f"chol_pairs1_{name}.npz"))
        b = np.load(os.path.join(scratch, f"chol_pairs0_{name}.npz"))
        same = all(np.array_equal(a[k], b[k]) for k in a.files)
        dev = max(float(np.max(np.abs(a[k] - b[k])) / max(np.max(np.abs(b[k])), 1e-300)) for k in a.files)
        print(json.dumps({"switch": env_name, "case": name, "K": K, "M": N, "bit_identical": same, "max_rel_dev": dev,
                          "prepare_ms_on": times["1"][name], "prepare_ms_off": times["0"][name]}))
    shutil.rmtree(scratch, ignore_errors=True)


if __name__ == "__main__":
    sys.exit(main())
