"""Device EM fit (gmm_cplx_bussgang.py:96-163, :437-790).

CPU: the oracle's M-step restatement against the reference's own estimate_gaussian_parameters
(tests/golden/fit.npz, made by make_golden_fit.py).  GPU: qce_em_mstep / qce_em_estep through the
C ABI against the same vectors and the oracle at larger shapes, and Gmm_nbit.fit end to end against
the reference's fitted models (same sklearn K-means initialisation, then device EM)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, rel_fro

FIX = os.path.join(GOLDEN, "fit.npz")


@pytest.fixture(scope="module")
def fx():
    return dict(np.load(FIX, allow_pickle=False))


def test_oracle_mstep_matches_reference(fx):
    from oracle import qce_oracle as O
    X, R = fx["h16"], fx["mstep_resp"]
    nk, mu, cov = O.em_mstep(X, R, 1e-6, "full", False)
    assert np.allclose(nk, fx["mstep_nk"], rtol=1e-13, atol=0)
    assert rel_fro(mu, fx["mstep_means"]) < 1e-13 and rel_fro(cov, fx["mstep_covs"]) < 1e-13
    _, _, cd = O.em_mstep(X, R, 1e-6, "diag", False)
    assert rel_fro(cd, fx["mstep_diag"]) < 1e-13
    _, mu0, cov0 = O.em_mstep(X, R, 1e-6, "full", True)
    assert not mu0.any() and rel_fro(cov0, fx["mstep_covs_zm"]) < 1e-13


def test_fit_rejects_unknown_covariance_type_without_device_work():
    from quantized_channel_estimation_amd import Gmm_nbit
    g = Gmm_nbit(n_components=2, covariance_type="tied")
    with pytest.raises(NotImplementedError):
        g.fit(np.zeros((10, 4), complex))


# ----------------------------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_gpu_mstep_matches_reference(fx):
    from quantized_channel_estimation_amd import _em
    X, R = fx["h16"], fx["mstep_resp"]
    em = _em.DeviceEM(X, R.shape[1], "full", 1e-6, False)
    nk, mu, cov = em.mstep(R)
    assert np.allclose(nk, fx["mstep_nk"], rtol=1e-12, atol=0)
    assert rel_fro(mu, fx["mstep_means"]) < 1e-12 and rel_fro(cov, fx["mstep_covs"]) < 1e-12
    emd = _em.DeviceEM(X, R.shape[1], "diag", 1e-6, False)
    _, _, cd = emd.mstep(R)
    assert rel_fro(cd, fx["mstep_diag"].real) < 1e-12
    em0 = _em.DeviceEM(X, R.shape[1], "full", 1e-6, True)
    _, mu0, cov0 = em0.mstep(R)
    assert not mu0.any() and rel_fro(cov0, fx["mstep_covs_zm"]) < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("B,N,K", [(5000, 64, 8), (3001, 48, 5), (700, 200, 3), (64, 16, 1), (9, 7, 2)])
def test_gpu_mstep_vs_oracle_shapes(B, N, K):
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import _em
    rng = np.random.default_rng(B + N + K)
    X = rng.standard_normal((B, N)) + 1j * rng.standard_normal((B, N)) + 0.3
    R = rng.random((B, K))
    R /= R.sum(axis=1, keepdims=True)
    for zm in (False, True):
        nk, mu, cov = _em.DeviceEM(X, K, "full", 1e-6, zm).mstep(R)
        nko, muo, covo = O.em_mstep(X, R, 1e-6, "full", zm)
        assert np.allclose(nk, nko, rtol=1e-12, atol=0)
        if not zm:
            assert rel_fro(mu, muo) < 1e-12
        assert rel_fro(cov, covo) < 1e-12, (B, N, K, zm)
        _, _, cd = _em.DeviceEM(X, K, "diag", 1e-6, zm).mstep(R)
        assert rel_fro(cd, O.em_mstep(X, R, 1e-6, "diag", zm)[2].real) < 1e-12


@pytest.mark.gpu
def test_gpu_estep_vs_oracle(golden_models):
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import _em
    m = golden_models["fullmean"]
    rng = np.random.default_rng(4)
    X = rng.standard_normal((1500, 32)) * 0.5 + 1j * rng.standard_normal((1500, 32)) * 0.5
    em = _em.DeviceEM(X, m["covs_cplx"].shape[0], "full", 1e-6, False)
    lb = em.estep(m["means_cplx"], m["covs_cplx"], m["weights"])
    P = O.precision_cholesky(m["covs_cplx"])
    norm, log_resp = O.log_prob_resp(X, m["means_cplx"], P, m["weights"])
    assert abs(lb - norm.mean()) <= 1e-10 * abs(norm.mean())
    R = em.R.cpu().numpy()
    assert np.abs(R - np.exp(log_resp)).max() < 1e-10
    assert np.array_equal(em.labels(), log_resp.argmax(axis=1))


def _kw(fx, tag):
    p = tag + "__kw_"
    out = {}
    for k in fx:
        if k.startswith(p):
            v = fx[k]
            out[k[len(p):]] = v.item() if v.ndim == 0 else v
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["full_zm", "full_mean", "full_rand", "circ", "bcirc", "full_ninit", "toep", "btoep"])
def test_gpu_fit_matches_reference(fx, tag):
    import warnings
    from quantized_channel_estimation_amd import Gmm_nbit
    p = tag + "__"
    ct = str(fx[p + "cov_type"])
    blocks = tuple(int(v) for v in fx[p + "blocks"])
    from threadpoolctl import threadpool_limits
    g = Gmm_nbit(covariance_type=ct, **_kw(fx, tag))
    with warnings.catch_warnings(), threadpool_limits(limits=1):  # deterministic K-means (make_golden_fit.py)
        warnings.simplefilter("ignore")
        g.fit(fx["h16"], blocks=blocks if blocks[0] else None, zero_mean=bool(fx[p + "zero_mean"]))
    info = (g.gm.n_iter_, g.gm.lower_bound_, float(fx[p + "lower_bound"]))
    # The inverse EM (toeplitz, :792-826) subtracts nearly equal terms (Cinv S Cinv - Cinv, cond(C) ~ 6e6
    # here): the reference's own arithmetic moves its lower bound by 2.6e-5 when np.linalg.pinv is
    # replaced by np.linalg.inv (measured, same data), so its bar is set at that scale.
    inv_em = "toep" in tag
    t_lb, t_par, t_chol = (2e-5, 1e-3, 1e-2) if inv_em else (1e-8, 1e-7, 1e-5)
    assert g.gm.n_iter_ == int(fx[p + "n_iter"]), info
    assert bool(g.gm.converged_) == bool(fx[p + "converged"]), info
    assert abs(g.gm.lower_bound_ - float(fx[p + "lower_bound"])) <= t_lb * max(1.0, abs(float(fx[p + "lower_bound"]))), info
    assert rel_fro(g.gm.weights_, fx[p + "weights"]) < t_par
    assert rel_fro(g.means_cplx, fx[p + "means_cplx"]) < 10 * t_par or np.abs(fx[p + "means_cplx"]).max() < 1e-12
    assert rel_fro(g.covs_cplx, fx[p + "covs_cplx"]) < t_par
    assert rel_fro(g.chol, fx[p + "chol"]) < t_chol
    if (p + "Sigma") in fx:
        assert rel_fro(g.gm.Sigma, fx[p + "Sigma"]) < t_par
    if (p + "fft_covs") in fx:
        assert rel_fro(g.fft_covs, fx[p + "fft_covs"].real) < 1e-7
    assert g.gm.covariance_type == "full"


@pytest.mark.gpu
def test_gpu_fit_then_estimate(fx):
    """A device-fitted model drops into estimate_from_y (the script's train-then-evaluate flow)."""
    import warnings
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import Gmm_nbit, observe
    h = fx["h16"]
    g = Gmm_nbit(n_components=6, covariance_type="full", random_state=0, max_iter=12)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        g.fit(h[:1000], zero_mean=True)
    y = observe.get_observation_nbit(h[1000:], 5.0, None, 1, seed=3)
    he = g.estimate_from_y(y, 5.0, 16, None, "all", 1)
    ho = O.estimate(g.means_cplx, g.covs_cplx, g.gm.weights_, y, 5.0, 16, None, "all", 1)
    assert rel_fro(he, ho) < 1e-5
