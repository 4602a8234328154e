"""Statistical achievable-rate lower bound (Bussgang_GMM.py:146-162 and copies).

The bound is inline script code (nothing importable to run on fixed inputs), so the oracle restates
those lines (oracle.rate_bound) and the GPU path is checked against it; the Bussgang pair it takes comes
from the estimate path's own pinned tables (K=1 model, Cr and gains = get_Cr / get_Bussgang_matrix for
1 bit and inf)."""
import numpy as np
import pytest


def _data(B=3000, N=32, seed=0):
    rng = np.random.default_rng(seed)
    h = (rng.standard_normal((B, N)) + 1j * rng.standard_normal((B, N))) * np.sqrt(0.5)
    he = h + 0.3 * (rng.standard_normal((B, N)) + 1j * rng.standard_normal((B, N)))
    A = rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N))
    cov = A @ A.conj().T / N + np.eye(N)
    return h, he, cov


def test_oracle_rate_is_finite_and_ordered():
    from oracle import qce_oracle as O
    h, he, cov = _data()
    g = np.full(32, 0.5)
    Cq = 0.1 * np.eye(32)
    r_est = O.rate_bound(he, h, g, Cq)[0]
    r_perfect = O.rate_bound(h, h, g, Cq)[0]
    assert np.isfinite(r_est) and r_perfect > r_est


@pytest.mark.gpu
@pytest.mark.parametrize("n_bits,clip", [(1, None), (1, 0.1), (np.inf, None)])
def test_gpu_rate_bound_vs_oracle(n_bits, clip):
    import torch
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import rate
    h, he, cov = _data()
    g, Cq, _ = rate.bussgang_global(cov, 5.0, n_bits)
    # the pair the scripts build (uniform_quantizer.get_Bussgang_matrix / get_Cr), restated
    Cy = cov + 10 ** (-5.0 / 10) * np.eye(32)
    if n_bits == 1:
        d = np.real(np.diag(Cy))
        gr = np.sqrt(2 / np.pi) / np.sqrt(d)
        P = np.diag(1 / np.sqrt(d))
        Cr = 2 / np.pi * (np.arcsin(np.clip(P @ Cy.real @ P, -1, 1)) + 1j * np.arcsin(np.clip(P @ Cy.imag @ P, -1, 1)))
    else:
        gr, Cr = np.ones(32), Cy
    assert np.allclose(g, gr, rtol=1e-13)
    assert np.abs(Cq - (Cr - np.diag(gr) @ cov @ np.diag(gr))).max() < 1e-12
    r, terms = rate.statistical_rate_bound(he, h, g, Cq, norm_clip=clip, return_terms=True)
    ro, num, den1, den2 = O.rate_bound(he, h, g, Cq, norm_clip=clip)
    assert abs(r - ro) <= 1e-11 * abs(ro)
    assert abs(terms["num"] - num) <= 1e-11 * num and abs(terms["den1"] - den1) <= 1e-10 * den1
    assert abs(terms["den2"] - den2) <= 1e-11 * den2
    rd = rate.statistical_rate_bound(torch.from_numpy(he).cuda(), torch.from_numpy(h).cuda(), g, Cq, norm_clip=clip)
    assert abs(rd - r) <= 1e-13 * abs(r)


@pytest.mark.gpu
@pytest.mark.parametrize("tag,snr,nb,qt", [("r2u", 5.0, 2, "uniform"), ("r3l", 0.0, 3, "lloyd"), ("r1", 5.0, 1, "uniform")])
def test_gpu_bussgang_pair_matches_reference(tag, snr, nb, qt):
    """get_Bussgang_matrix / get_Cr of the reference (tests/golden/baselines.npz) for the rate bound."""
    import os
    from conftest import GOLDEN
    from quantized_channel_estimation_amd import inputs, rate
    bl = np.load(os.path.join(GOLDEN, "baselines.npz"), allow_pickle=False)
    quantizer = inputs.get_quantizer([snr], nb, qt)[snr]
    g, Cq, Cr = rate.bussgang_global(bl["C"], snr, nb, quantizer)
    assert np.abs(g - bl[tag + "__buss"]).max() <= 1e-13 * np.abs(g).max()
    assert np.abs(Cr - bl[tag + "__Cr"]).max() <= 1e-11 * np.abs(Cr).max()


def test_quantized_variance_matches_reference():
    import os
    from conftest import GOLDEN
    from quantized_channel_estimation_amd import inputs, rate
    bl = np.load(os.path.join(GOLDEN, "baselines.npz"), allow_pickle=False)
    for tag, snr, nb, qt in [("r2u", 5.0, 2, "uniform"), ("r3l", 0.0, 3, "lloyd")]:
        quantizer = inputs.get_quantizer([snr], nb, qt)[snr]
        d = np.real(np.diag(bl["C"])) + 10 ** (-snr / 10)
        assert np.allclose(rate.quantized_variance(d, quantizer[0], quantizer[1]), np.real(np.diag(bl[tag + "__Cr"])),
                           rtol=1e-12, atol=0)


def test_oracle_mf_rate_is_finite_and_ordered():
    from oracle import qce_oracle as O
    h, he, cov = _data(B=200)
    g = np.full(32, 0.5)
    Cq = 0.1 * np.eye(32) + 0.02 * cov
    r_est = O.rate_mf(he, h, g, Cq)
    r_perfect = O.rate_mf(h, h, g, Cq)
    assert np.isfinite(r_est) and r_perfect > r_est


@pytest.mark.gpu
@pytest.mark.parametrize("n_bits", [1, np.inf])
def test_gpu_mf_rate_vs_oracle(n_bits):
    """LS branch per-sample rate (Bussgang_GMM.py:186-198) on the device vs the loop restatement."""
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import rate
    h, he, cov = _data(B=500)
    g, Cq, _ = rate.bussgang_global(cov, 5.0, n_bits)
    r = rate.matched_filter_rate(he, h, g, Cq)
    ro = O.rate_mf(he, h, g, Cq)
    assert np.isfinite(r) and abs(r - ro) <= 1e-9 * abs(ro)


@pytest.mark.gpu
def test_gpu_mf_rate_ill_conditioned_cq_and_not_pd():
    """Cq^-1 of the matched-filter rate is eliminated from [Cq | I] directly (no Cq^H Cq, so cond(Cq) is
    not squared): an ill-conditioned Cq (cond 1e6) matches the loop restatement; an indefinite Cq raises."""
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import rate
    h, he, _ = _data(B=200)
    N = h.shape[1]
    rng = np.random.default_rng(3)
    Q, _ = np.linalg.qr(rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N)))
    Cq = Q @ np.diag(np.logspace(0, -6, N)) @ Q.conj().T
    Cq = 0.5 * (Cq + Cq.conj().T)
    g = np.full(N, np.sqrt(2 / np.pi))
    r = rate.matched_filter_rate(he, h, g, Cq)
    ro = O.rate_mf(he, h, g, Cq)
    assert np.isfinite(r) and abs(r - ro) <= 1e-6 * abs(ro)
    Cbad = Cq.copy()
    Cbad[0, 0] = -1.0
    with pytest.raises(ValueError, match="positive definite"):
        rate.matched_filter_rate(he, h, g, Cbad)
