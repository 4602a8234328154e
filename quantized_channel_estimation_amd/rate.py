"""Achievable-rate lower bound of the experiment scripts on the device (SURVEY.md §8(f) row 4;
reference Bussgang_GMM.py:146-162, :206-216, :238-249, :291-306 — inline script code, restated here):
``statistical_rate_bound`` runs ``qce_rate_bound`` (csrc/qce_rate.hip).  ``bussgang_global`` gives the
(B, Cq) pair the scripts build from the global sample covariance (get_Bussgang_matrix / get_Cr,
uniform_quantizer.py:60-73, :114-173): gains and Cy from a one-component device model; for multi-bit
quantisers get_Cr's diagonal is the quantiser's output variance (an N-vector of Gaussian-CDF sums,
evaluated here on the host as part of the per-SNR setup).
"""
import numpy as np

from . import _lib


def statistical_rate_bound(h_est, h, buss, Cq, norm_clip=None, device=0, return_terms=False):
    """log2(1 + |mean g^H B h|^2 / (var(g^H B h) + mean g^H Cq g)), g = h_est / ||h_est||^2."""
    buss = np.ascontiguousarray(np.real(np.diag(buss)) if np.ndim(buss) == 2 else np.real(buss), dtype=np.float64)
    Cq = np.ascontiguousarray(Cq, dtype=np.complex128)
    out = np.zeros(4)
    if hasattr(h_est, "data_ptr") and not isinstance(h_est, np.ndarray):
        import torch
        a = h_est.to(torch.complex128).contiguous()
        b = h.to(torch.complex128).contiguous()
        torch.cuda.current_stream(a.device).synchronize()
        B, N = a.shape
        _lib.check(_lib.load().qce_rate_bound(_lib.ptr(a), _lib.ptr(b), B, N, _lib.ptr(buss), _lib.ptr(Cq),
                                              float(norm_clip or 0.0), _lib.ptr(out), a.device.index or 0,
                                              _lib.IO_DEVICE, None))
    else:
        a = np.ascontiguousarray(h_est, dtype=np.complex128)
        b = np.ascontiguousarray(h, dtype=np.complex128)
        B, N = a.shape
        _lib.check(_lib.load().qce_rate_bound(_lib.ptr(a), _lib.ptr(b), B, N, _lib.ptr(buss), _lib.ptr(Cq),
                                              float(norm_clip or 0.0), _lib.ptr(out), int(device), _lib.IO_HOST,
                                              None))
    if return_terms:
        return float(out[0]), dict(num=float(out[1]), den1=float(out[2]), den2=float(out[3]))
    return float(out[0])


def matched_filter_rate(h_est, h, buss, Cq, device=0):
    """Per-sample matched-filter rate of the LS branch (Bussgang_GMM.py:186-198), averaged over samples:
    g = h_est_b^H B^H Cq^-1, Re log2(1 + |g B h_est_b|^2 / (g Cq g^H + |g B (h_b - h_est_b)|^2))."""
    buss = np.ascontiguousarray(np.real(np.diag(buss)) if np.ndim(buss) == 2 else np.real(buss), dtype=np.float64)
    Cq = np.ascontiguousarray(Cq, dtype=np.complex128)
    a = np.ascontiguousarray(h_est, dtype=np.complex128)
    b = np.ascontiguousarray(h, dtype=np.complex128)
    B, N = a.shape
    out = np.zeros(1)
    _lib.check(_lib.load().qce_rate_mf(_lib.ptr(a), _lib.ptr(b), B, N, _lib.ptr(buss), _lib.ptr(Cq), _lib.ptr(out),
                                       int(device), _lib.IO_HOST, None))
    return float(out[0])


def quantized_variance(d, thresholds, labels):
    """get_quantized_variance (uniform_quantizer.py:114-128): output variance of the per-component
    quantiser for complex inputs of variance d."""
    from scipy.special import ndtr
    s = np.sqrt(np.asarray(d, dtype=float) / 2)[:, None]
    thr = np.asarray(thresholds, dtype=float)[None, :]
    lab = np.asarray(labels, dtype=float)
    cdf = ndtr(thr / s)
    res = lab[0] ** 2 * cdf[:, 0] + lab[-1] ** 2 * (1 - cdf[:, -1])
    res = res + (lab[1:-1] ** 2 * (cdf[:, 1:] - cdf[:, :-1])).sum(axis=1)
    return 2 * res


def bussgang_global(cov, snr, n_bits, quantizer=None, device=0):
    """(diag Bussgang gain (N,), Cq = Cr - B C B^H) of Cy = cov + 10^(-snr/10) I (the scripts' Cy_act,
    Bussgang_GMM.py:148-151): uniform-quantiser gains (the scripts call uniform_quantizer's functions for
    every quantiser type); multi-bit Cr = mean(gain)^2 Cy with the quantised variance of
    ``quantizer = (thresholds, labels, _)`` on the diagonal (get_Cr, :165-171)."""
    nb = float(n_bits)
    cov = np.asarray(cov, dtype=complex)
    dm = _lib.DeviceModel(None, cov[None], np.ones(1), device=device)
    try:
        dm.prepare(None, snr, nb, _lib.QUANT_UNIFORM)
        t = dm.tables()
    finally:
        dm.close()
    g = np.real(np.diag(t["A_eff"][0]))
    if nb == 1.0 or np.isinf(nb):
        Cr = t["Cr"][0]
    else:
        if quantizer is None or quantizer[0] is None:
            raise ValueError("multi-bit get_Cr needs the quantizer (thresholds, labels, rho)")
        Cy = t["Cy"][0]
        Cr = np.mean(g) ** 2 * Cy
        np.fill_diagonal(Cr, quantized_variance(np.real(np.diag(Cy)), quantizer[0], quantizer[1]))
    Cq = Cr - (g[:, None] * cov) * g[None, :]
    return g, Cq, Cr
