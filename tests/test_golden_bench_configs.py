"""Parity at the BASELINE.json configurations' model sizes against the reference itself
(tests/golden/bench_configs.npz, made by tests/golden/make_golden_bench.py from the reference's own
Gmm_nbit.estimate_from_y): K = 16..256, N = 32..256, full / circulant / block-circulant covariances, 1-bit,
2-bit uniform and 3-bit Lloyd-Max quantisers, zero-mean and with means; 64 observations per configuration.

The CPU tests pin the oracle there (FP64 against FP64: 1e-10); the GPU tests run the drop-in
`Gmm_nbit.estimate_from_y` on the HIP path (north_star bar 1e-5, the FP64 kernels land near 1e-13; labels exact)."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT, rel_fro

sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from make_golden_bench import CASES, checksum, model_of  # noqa: E402

FX = os.path.join(ROOT, "tests", "golden", "bench_configs.npz")
TAGS = [n + s for n in CASES for s in ("", "_mean")]


@pytest.fixture(scope="module")
def fx():
    return dict(np.load(FX))


def _case(fx, tag):
    base = tag[:-5] if tag.endswith("_mean") else tag
    c = CASES[base]
    means, covs, w = model_of(c, tag.endswith("_mean"))
    np.testing.assert_allclose(checksum(means, covs, w), fx[tag + "__checksum"], rtol=1e-12, atol=1e-12,
                               err_msg="the bench model recipe changed since the fixture was made")
    p = base + "__"
    qz = (fx[p + "thr"], fx[p + "lab"], None) if (p + "thr") in fx else (None, None, None)
    return c, means, covs, w, fx[p + "y"], qz


@pytest.mark.parametrize("tag", TAGS)
def test_oracle_matches_reference_at_bench_sizes(fx, tag):
    from oracle import qce_oracle as O
    c, means, covs, w, y, qz = _case(fx, tag)
    args = (y, c["snr"], c["N"], None)
    tail = (c["n_bits"], c["qtype"], qz)
    h = O.estimate(means, covs, w, *args, "all", *tail)
    assert rel_fro(h, fx[tag + "__hest_all"]) < 1e-10, rel_fro(h, fx[tag + "__hest_all"])
    h1 = O.estimate(means, covs, w, *args, 1, *tail)
    assert rel_fro(h1, fx[tag + "__hest_top1"]) < 1e-10, rel_fro(h1, fx[tag + "__hest_top1"])


@pytest.mark.gpu
@pytest.mark.parametrize("tag", TAGS)
def test_hip_path_matches_reference_at_bench_sizes(fx, tag):
    from quantized_channel_estimation_amd import Gmm_nbit, _lib
    if _lib.device_count() == 0:
        pytest.fail("no GPU visible for a gpu-marked test")
    c, means, covs, w, y, qz = _case(fx, tag)
    g = Gmm_nbit.from_params(means, covs, w)
    args = (c["snr"], c["N"], None)
    tail = (c["n_bits"], c["qtype"], qz)
    h = g.estimate_from_y(y, *args, "all", *tail)
    err = rel_fro(h, fx[tag + "__hest_all"])
    assert err < 1e-9, (tag, err)
    np.testing.assert_array_equal(g._predict_cplx(y), fx[tag + "__labels"])
    h1 = g.estimate_from_y(y, *args, 1, *tail)
    assert rel_fro(h1, fx[tag + "__hest_top1"]) < 1e-9, (tag, rel_fro(h1, fx[tag + "__hest_top1"]))
    print(tag, "rel err", err, "structure", g._dev.structure())
