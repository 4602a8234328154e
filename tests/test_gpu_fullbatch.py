"""Every BASELINE.json GPU configuration at its FULL batch size (bench.py's inputs: SCM channel pool, fresh noise,
the quantiser of the config), 'all' mode through the C-ABI with device I/O in one launch, checked against the FP64
oracle on row windows that cover the kernels' schedule boundaries: the first rows, the persistent grids' round
edges, the middle and the ragged end (the oracle's 'all' mode materialises rows x K x N filter outputs, so it runs
on windows, not the whole batch).  Size-independent property on the whole batch: every row finite, and the same
rows estimated as one small batch equal the full-batch rows (launch geometry is not arithmetic)."""
import os
import sys

import numpy as np
import pytest

from conftest import rel_fro

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu

F64_TOL = 1e-9


def _windows(B, edges, w=160):
    out = [(0, w), (B - w, B), (B // 2 - w // 2, B // 2 + w // 2)]
    for e in edges:
        lo = max(0, min(B - w, e - w // 2))
        out.append((lo, lo + w))
    return out


@pytest.mark.parametrize("config", ["metric", "cfg2", "cfg3", "cfg4", "cfg5"])
def test_full_batch_vs_oracle(config):
    import torch
    import bench
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import _lib
    cfg = dict(bench.CONFIGS[config])
    K, N, B = cfg["K"], cfg["N"], cfg["B"]
    means, covs, w, h, y, qz = bench.make_inputs(cfg, 0)
    dm = _lib.DeviceModel(means, covs, w)
    kind = _lib.QUANT_LLOYD if cfg.get("qtype") == "lloyd" else _lib.QUANT_UNIFORM
    dm.prepare(None, cfg["snr"], float(cfg["n_bits"]), kind, qz[0], qz[1])
    assert bool(dm.structure()[2]) == (cfg["cov"] != "full")
    yd = torch.from_numpy(y).to("cuda")
    hg = dm.estimate(yd)
    hg = hg.cpu().numpy() if hasattr(hg, "cpu") else np.asarray(hg)
    assert hg.shape == (B, N) and np.isfinite(hg).all()
    # schedule edges: 16-row tiles x (2 workgroups x 4 waves x 256 CUs) for the Fourier kernels' persistent rounds,
    # 128-row tiles x 256 workgroups for the dense kernel's whole rounds
    edges = [2048 * 16, 4096 * 16, 256 * 128, 512 * 128, (B // (256 * 128)) * 256 * 128]
    edges = [e for e in edges if 0 < e < B]
    rows = []
    for lo, hi in _windows(B, edges):
        ho = O.estimate(means, covs, w, y[lo:hi], cfg["snr"], N, None, "all", cfg["n_bits"], cfg["qtype"], qz)
        err = rel_fro(hg[lo:hi], ho)
        assert err < F64_TOL, (config, lo, hi, err)
        rows.append(np.arange(lo, hi))
    # the same rows estimated as a small batch give the same values (launch geometry is not arithmetic)
    sel = np.concatenate(rows)
    hs = dm.estimate(torch.from_numpy(np.ascontiguousarray(y[sel])).to("cuda"))
    hs = hs.cpu().numpy() if hasattr(hs, "cpu") else np.asarray(hs)
    assert rel_fro(hs, hg[sel]) < 1e-12
    dm.close()
