"""Adopting reference-fitted models (the scripts' joblib path, Bussgang_GMM.py:270-278) and the state-mirror
lifecycle across estimate -> fit -> pickle (pool.starmap, :282-287)."""
import copy
import os
import pickle

import numpy as np
import pytest

from conftest import GOLDEN, MODES, case_args, load_model, rel_fro

pytestmark = pytest.mark.gpu


class _RefLike:
    """Duck-typed stand-in for a joblib-loaded reference Gmm_nbit: the attributes the estimate path reads
    (means_cplx, covs_cplx, gm.weights_ / covariance_type / n_components, params)."""

    def __init__(self, fx):
        from sklearn.mixture import GaussianMixture
        K = int(fx["K"])
        self.gm = GaussianMixture(n_components=K, covariance_type="full")
        self.gm.weights_ = np.array(fx["weights"])
        self.means_cplx = np.array(fx["means_cplx"])
        self.covs_cplx = np.array(fx["covs_cplx"])
        self.params = {"zero_mean": not np.any(self.means_cplx)}


@pytest.mark.parametrize("mname", ["full", "fullmean", "circ"])
def test_gmm_from_reference_matches_golden(mname):
    from quantized_channel_estimation_amd import Gmm_nbit
    fx = load_model(mname)
    ref = _RefLike(fx)
    g = Gmm_nbit.from_reference(ref)
    assert g.gm is not ref.gm and g.covs_cplx is not ref.covs_cplx  # deep copies, as the scripts' deepcopy
    tag = str(fx["cases"][0])
    y, snr, N, A, n_bits, qtype, quantizer = case_args(fx, tag)
    # Fourier-domain path at 1 bit: the reference's entry-wise arcsine law on its dense Cy amplifies last-bit
    # differences (the documented sensitivity of tests/test_gpu_parity.py), so h 1e-7 and proba 1e-4 there
    fourier1 = mname in ("circ", "bcirc") and n_bits == 1
    for mtag, mode in MODES.items():
        h = g.estimate_from_y(y, snr, N, A, mode, n_bits, qtype, quantizer)
        assert rel_fro(h, fx[f"{tag}__hest_{mtag}"]) < (1e-7 if fourier1 else 1e-9), (mname, mtag)
    np.testing.assert_allclose(g.predict_proba_cplx(y), fx[f"{tag}__proba"], rtol=1e-4 if fourier1 else 1e-8,
                               atol=1e-12)
    # the reference's object is untouched (the adoption copies)
    assert not hasattr(ref.gm, "means_") or ref.gm.means_ is None


def test_mofa_from_reference_matches_golden():
    from quantized_channel_estimation_amd import Mofa
    mf = dict(np.load(os.path.join(GOLDEN, "mofa.npz"), allow_pickle=False))

    class RefMofa:
        pass
    r = RefMofa()
    K, D, M = mf["lambdas"].shape
    r.n_components, r.M, r.D = K, M, D
    r.means, r.covs, r.amps, r.lambdas, r.psis = mf["means"], mf["covs"], mf["amps"], mf["lambdas"], mf["psis"]
    r.zero_mean = not np.any(mf["means"])
    m = Mofa.from_reference(r)
    y, snr = mf["b1__y"], float(mf["b1__snr"])
    for name, mode in (("all", "all"), ("top1", 1)):
        h = m.estimate_from_y(y, snr, None, mode, 1, "uniform", (None, None, None))
        assert rel_fro(h, mf[f"b1__h_{name}"]) < 1e-9, name


def test_estimate_then_fit_then_pickle_keeps_fitted_state():
    """an estimate leaves the observation-domain state pending; a later fit must not be overwritten
    by it when the object is pickled (pool.starmap) or deep-copied."""
    from quantized_channel_estimation_amd import Gmm_nbit, inputs
    rng = np.random.default_rng(3)
    N = 16
    h1, _ = inputs.scm_generate(800, 1, N, rng, n_path=3)
    h2, _ = inputs.scm_generate(800, 1, N, rng, n_path=3)
    h1, h2 = h1[:, 0, :].astype(complex), h2[:, 0, :].astype(complex)
    g = Gmm_nbit(n_components=3, covariance_type="full", max_iter=5, random_state=0)
    g.fit(h1, zero_mean=True)
    y = inputs.get_observation_nbit(h1[:64], 5.0, None, 1, rng=rng)
    g.estimate_from_y(y, 5.0, N, None, "all", 1)
    assert "_qce_pending" in g.gm.__dict__
    g.fit(h2, zero_mean=True)
    fitted = (np.array(g.gm.means_), np.array(g.gm.covariances_))
    for obj in (pickle.loads(pickle.dumps(g)), copy.deepcopy(g)):
        np.testing.assert_array_equal(obj.gm.means_, fitted[0])
        np.testing.assert_array_equal(obj.gm.covariances_, fitted[1])


def test_frozen_params_skip_digest_and_inplace_edits_still_seen():
    """Writeable parameters are re-digested every call (in-place edits take effect, as in the reference);
    freeze_params() makes the digest reusable while the same read-only arrays are attached."""
    from quantized_channel_estimation_amd import Gmm_nbit, gmm
    fx = load_model("full")
    tag = str(fx["cases"][0])
    y, snr, N, A, n_bits, qtype, quantizer = case_args(fx, tag)
    g = Gmm_nbit.from_params(fx["means_cplx"], np.array(fx["covs_cplx"]), fx["weights"])
    h0 = g.estimate_from_y(y, snr, N, A, "all", n_bits, qtype, quantizer)
    g.covs_cplx[0] *= 2.0  # in-place edit of a writeable array: the next estimate must see it
    h1 = g.estimate_from_y(y, snr, N, A, "all", n_bits, qtype, quantizer)
    assert rel_fro(h1, h0) > 1e-6
    g.freeze_params()
    calls = {"n": 0}
    orig = gmm._fingerprint

    def counting(*a):
        calls["n"] += 1
        return orig(*a)
    gmm._fingerprint = counting
    try:
        for _ in range(3):
            h2 = g.estimate_from_y(y, snr, N, A, "all", n_bits, qtype, quantizer)
    finally:
        gmm._fingerprint = orig
    assert calls["n"] == 1
    assert rel_fro(h2, h1) < 1e-14
