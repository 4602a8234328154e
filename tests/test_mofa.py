"""MFA Bussgang estimator (mofa_cplx_bussgang.py:117-216, :342-368).

CPU: the oracle (the GMM restatement fed with C_k = Lambda Lambda^H + Psi and the amps) reproduces
the reference Mofa's estimates in tests/golden/mofa.npz (made by make_golden_mofa.py from the
reference itself).  GPU: quantized_channel_estimation_amd.Mofa through libqce.so against the same
vectors: h within 1e-5 relative Frobenius, argmax labels exact."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, rel_fro

MODES = {"all": "all", "top1": 1, "top3": 3, "p09": 0.9}


@pytest.fixture(scope="module")
def mf():
    return dict(np.load(os.path.join(GOLDEN, "mofa.npz"), allow_pickle=False))


def _case(mf, tag):
    p = tag + "__"
    nb = float(mf[p + "n_bits"])
    quantizer = (mf[p + "thr"], mf[p + "lab"], None) if (p + "thr") in mf else (None, None, None)
    return mf[p + "y"], float(mf[p + "snr"]), (np.inf if np.isinf(nb) else int(nb)), str(mf[p + "qtype"]), quantizer


def test_factor_covariances(mf):
    from quantized_channel_estimation_amd import Mofa
    m = Mofa.from_params(mf["means"], mf["lambdas"], mf["psis"], mf["amps"])
    assert rel_fro(m.covs, mf["covs"]) < 1e-13


@pytest.mark.parametrize("tag", ["b1", "b2u", "b3l", "inf"])
def test_oracle_matches_reference_mofa(mf, tag):
    from oracle import qce_oracle as O
    y, snr, nb, qt, quantizer = _case(mf, tag)
    N = mf["covs"].shape[-1]
    for name, mode in MODES.items():
        ho = O.estimate(mf["means"], mf["covs"], mf["amps"], y, snr, N, None, mode, nb, qt, quantizer)
        assert rel_fro(ho, mf[f"{tag}__h_{name}"]) < 1e-9, (tag, name)


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["b1", "b2u", "b3l", "inf"])
def test_gpu_mofa_matches_reference(mf, tag):
    from quantized_channel_estimation_amd import Mofa
    m = Mofa.from_params(mf["means"], mf["lambdas"], mf["psis"], mf["amps"])
    y, snr, nb, qt, quantizer = _case(mf, tag)
    for name, mode in MODES.items():
        h = m.estimate_from_y(y, snr, None, mode, nb, qt, quantizer)
        assert h.dtype == y.dtype
        assert rel_fro(h, mf[f"{tag}__h_{name}"]) < 1e-5, (tag, name)
    pr = m.predict_proba(y)  # observation-domain model after the estimate, as the reference
    assert np.abs(pr - mf[f"{tag}__proba_obs"]).max() < 1e-6
    assert np.array_equal(m.predict_proba_max(y), mf[f"{tag}__proba_obs"].argmax(axis=1))


@pytest.mark.gpu
def test_gpu_mofa_channel_domain_proba(mf):
    from quantized_channel_estimation_amd import Mofa
    m = Mofa.from_params(mf["means"], mf["lambdas"], mf["psis"], mf["amps"])
    pr = m.predict_proba(mf["h_val"][:50])
    assert np.abs(pr - mf["proba_chan"]).max() < 1e-6
