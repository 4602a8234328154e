"""MFA EM (quantized_channel_estimation_amd.Mofa.fit; reference mofa_cplx_bussgang.py:94-115, :219-338,
:404-422) against tests/golden/mofa_fit.npz, made by make_golden_mofa_fit.py from the reference's own
_initialize and run_em (three cases: zero mean; with means; PPCA + lock_psis).

Parity is held per EM step (from the reference's parameters before iteration i, one step gives its
parameters before iteration i+1 and its lower bound L_i) and for the whole fit (init -> final parameters,
L_all): the moment form reorders the reference's sums, which moves the trajectory by ~1e-12 over a dozen
iterations on the CPU.

CPU: the initialisation reproduces the reference's draws from numpy's global RNG; the host-side M-step
algebra (latent sums from the weighted moments) fed with NumPy moments reproduces every reference step.
GPU: the same steps with the E-step and the moments on the device, and the full fit."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, rel_fro


@pytest.fixture(scope="module")
def mf():
    return dict(np.load(os.path.join(GOLDEN, "mofa_fit.npz"), allow_pickle=False))


def _cfg(mf, tag):
    K, M, zm, ppca, lock, maxiter, seed = (int(v) for v in mf[tag + "__cfg"])
    return K, M, bool(zm), bool(ppca), bool(lock), maxiter, seed


def _init(mf, tag):
    p = tag + "__init_"
    return mf[p + "means"], mf[p + "lambdas"], mf[p + "psis"], mf[p + "amps"]


def _step_params(mf, tag, i):
    p = tag + "__it_"
    return mf[p + "means"][i], mf[p + "lambdas"][i], mf[p + "psis"][i], mf[p + "amps"][i]


def _check_step(mf, tag, i, got, L, tol):
    means, lambdas, psis, amps = got
    em, el, ep, ea = _step_params(mf, tag, i + 1)
    assert abs(L - mf[tag + "__L_all"][i]) <= tol * abs(mf[tag + "__L_all"][i]), (i, L)
    for name, g, e in (("lambdas", lambdas, el), ("psis", psis, ep), ("amps", amps, ea), ("means", means, em)):
        if np.abs(e).max() == 0:
            assert np.abs(g).max() == 0, name
        else:
            assert rel_fro(g, e) < tol, (i, name, rel_fro(g, e))


def _numpy_stats(data, zero_mean):
    from scipy.special import logsumexp
    from quantized_channel_estimation_amd.mofa import EPS10

    def stats(means, covs, amps):
        B, D = data.shape
        K = covs.shape[0]
        lp = np.empty((B, K))
        for k in range(K):
            x1 = data - means[k]
            _, ld = np.linalg.slogdet(covs[k])
            q = np.real(np.sum(x1.conj() * (x1 @ np.linalg.inv(covs[k]).T), axis=1))
            lp[:, k] = np.log(amps[k]) - D * np.log(np.pi) - ld - q
        lb = logsumexp(lp, axis=1)
        r = np.exp(lp - lb[:, None])
        s0 = r.sum(0)
        nk = s0 + EPS10
        mbar = np.zeros((K, D), complex) if zero_mean else (r.T @ data) / nk[:, None]
        qbar = np.stack([((r[:, k, None] * (data - mbar[k])).T @ (data - mbar[k]).conj()) for k in range(K)])
        d = r.T @ data - s0[:, None] * mbar
        return lb.sum(), s0, mbar, qbar, d
    return stats


@pytest.mark.parametrize("tag", ["zm", "mean", "ppca_lock"])
def test_initialize_reproduces_reference_draws(mf, tag):
    from threadpoolctl import threadpool_limits
    from quantized_channel_estimation_amd import Mofa
    K, M, zm, ppca, lock, maxiter, seed = _cfg(mf, tag)
    m = Mofa(K, M, PPCA=ppca, lock_psis=lock)
    m.zero_mean = zm
    np.random.seed(seed)
    with threadpool_limits(limits=1):
        got = m._initialize(mf["data"])
    for g, e in zip(got, _init(mf, tag)):
        np.testing.assert_allclose(g, e, rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("tag", ["zm", "mean", "ppca_lock"])
def test_em_fit_from_moments_matches_reference(mf, tag):
    from quantized_channel_estimation_amd.mofa import mfa_em
    K, M, zm, ppca, lock, maxiter, seed = _cfg(mf, tag)
    data = mf["data"]
    res = mfa_em(_init(mf, tag), _numpy_stats(data, zm), maxiter, 1e-14, zm, ppca, lock, data.shape[0])
    means, lambdas, psis, amps, covs, _, L_all, _ = res
    np.testing.assert_allclose(L_all, mf[tag + "__L_all"], rtol=1e-10)
    for name, v in (("lambdas", lambdas), ("psis", psis), ("amps", amps), ("covs", covs)):
        assert rel_fro(v, mf[tag + "__" + name]) < 1e-9, name


@pytest.mark.parametrize("tag", ["zm", "mean", "ppca_lock"])
def test_em_steps_from_moments_match_reference(mf, tag):
    from quantized_channel_estimation_amd.mofa import mfa_em
    K, M, zm, ppca, lock, maxiter, seed = _cfg(mf, tag)
    data = mf["data"]
    stats = _numpy_stats(data, zm)
    for i in range(len(mf[tag + "__L_all"])):
        res = mfa_em(_step_params(mf, tag, i), stats, 1, 1e-14, zm, ppca, lock, data.shape[0])
        _check_step(mf, tag, i, res[:4], res[6][0], 1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["zm", "mean", "ppca_lock"])
def test_gpu_mfa_em_steps_and_fit(mf, tag):
    from threadpoolctl import threadpool_limits
    from quantized_channel_estimation_amd import Mofa, _lib
    if _lib.device_count() == 0:
        pytest.fail("no GPU visible for a gpu-marked test")
    K, M, zm, ppca, lock, maxiter, seed = _cfg(mf, tag)
    data = mf["data"]
    L_ref = mf[tag + "__L_all"]
    for i in range(len(L_ref)):  # one device EM step from each of the reference's states
        m = Mofa(K, M, PPCA=ppca, lock_psis=lock, maxiter=1, tol=1e-14, verbose=False)
        m.fit(data, zero_mean=zm, init=_step_params(mf, tag, i))
        _check_step(mf, tag, i, (m.means, m.lambdas, m.psis, m.amps), m.L_all[0], 1e-8)
    # the whole fit from a seeded global RNG (the reference's initialisation)
    m2 = Mofa(K, M, PPCA=ppca, lock_psis=lock, maxiter=maxiter, tol=1e-14, verbose=False)
    np.random.seed(seed)
    with threadpool_limits(limits=1):
        m2.fit(data, zero_mean=zm)
    assert len(m2.L_all) == len(L_ref)
    np.testing.assert_allclose(m2.L_all, L_ref, rtol=1e-8)
    p = tag + "__"
    for name in ("lambdas", "psis", "amps", "covs"):
        assert rel_fro(getattr(m2, name), mf[p + name]) < 1e-7, name
    assert np.all(m2.psis >= 1e-6) and abs(m2.amps.sum() - 1) < 1e-12
    y = (np.sign(data[:64].real) + 1j * np.sign(data[:64].imag)) / np.sqrt(2)
    h = m2.estimate_from_y(y, 5.0, None, "all", 1)
    assert h.shape == (64, data.shape[1]) and np.isfinite(h).all()
