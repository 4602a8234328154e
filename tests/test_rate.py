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
    g, Cq = rate.bussgang_global(cov, 5.0, n_bits)
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
