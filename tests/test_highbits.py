"""Uniform quantisers beyond J. Max's table (n_bits 9..16): the reference's asymptotic step 4 sqrt(b) 2^-b
(uniform_quantizer.py:6-23, `else` at :15) in the quantiser tables and the Bussgang gain.  Pinned to
tests/golden/highbits.npz (tests/golden/make_golden_highbits.py, made by the reference itself)."""
import os
import warnings

import numpy as np
import pytest

from conftest import ROOT, rel_fro

HB = os.path.join(ROOT, "tests", "golden", "highbits.npz")


@pytest.fixture(scope="module")
def hb():
    return np.load(HB)


def _case(hb, tag):
    return (hb[tag + "__y"], float(hb[tag + "__snr"]), int(hb[tag + "__n_bits"]),
            (hb[tag + "__thr"], hb[tag + "__lab"], None))


def test_oracle_highbits(hb):
    from oracle import qce_oracle as O
    N = hb["covs_cplx"].shape[-1]
    for tag in hb["cases"]:
        tag = str(tag)
        y, snr, nb, qz = _case(hb, tag)
        for mtag, mode in (("all", "all"), ("top1", 1)):
            h = O.estimate(hb["means_cplx"], hb["covs_cplx"], hb["weights"], y, snr, N, None, mode, nb, "uniform", qz)
            assert rel_fro(h, hb[f"{tag}__hest_{mtag}"]) < 1e-11, (tag, mtag)


def test_quantizer_tables_highbits(hb):
    """The package's quantiser producer (inputs.get_quantizer, utils.py:531-562) beyond 8 bits."""
    from quantized_channel_estimation_amd import inputs
    for tag in hb["cases"]:
        tag = str(tag)
        _, snr, nb, (thr, lab, _) = _case(hb, tag)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            t2, l2, _ = inputs.get_quantizer([snr], nb, "uniform")[snr]
        np.testing.assert_allclose(t2, thr, rtol=1e-13, atol=1e-15)
        np.testing.assert_allclose(l2, lab, rtol=1e-13, atol=1e-15)


@pytest.mark.gpu
def test_device_highbits(hb):
    from quantized_channel_estimation_amd import Gmm_nbit
    N = hb["covs_cplx"].shape[-1]
    for tag in hb["cases"]:
        tag = str(tag)
        y, snr, nb, qz = _case(hb, tag)
        g = Gmm_nbit.from_params(hb["means_cplx"], hb["covs_cplx"], hb["weights"])
        for mtag, mode in (("all", "all"), ("top1", 1)):
            with pytest.warns(UserWarning, match="approximated"):
                h = g.estimate_from_y(y, snr, N, None, mode, nb, "uniform", qz)
            assert rel_fro(h, hb[f"{tag}__hest_{mtag}"]) < 1e-9, (tag, mtag, rel_fro(h, hb[f"{tag}__hest_{mtag}"]))
        np.testing.assert_allclose(g.gm.means_, hb[tag + "__means_y"], rtol=1e-10, atol=1e-13)


@pytest.mark.gpu
def test_device_nbits_beyond_limit():
    """Beyond 16 bits (2^b - 1 gain terms per diagonal entry) and Lloyd-Max beyond 8 bits: NotImplementedError."""
    from quantized_channel_estimation_amd import _lib
    rng = np.random.default_rng(0)
    N = 16
    X = rng.standard_normal((4, N, N)) + 1j * rng.standard_normal((4, N, N))
    covs = X @ X.conj().transpose(0, 2, 1) / N + np.eye(N)
    dm = _lib.DeviceModel(None, covs, np.full(4, 0.25))
    with pytest.raises(NotImplementedError):
        dm.prepare(None, 5.0, 17, _lib.QUANT_UNIFORM)
    with pytest.raises(NotImplementedError):
        dm.prepare(None, 5.0, 9, _lib.QUANT_LLOYD, np.zeros(511), np.zeros(512))
