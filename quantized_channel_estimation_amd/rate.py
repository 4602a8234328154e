"""Achievable-rate lower bound of the experiment scripts on the device (SURVEY.md §8(f) row 4;
reference Bussgang_GMM.py:146-162, :206-216, :238-249, :291-306 — inline script code, restated here):
``statistical_rate_bound`` runs ``qce_rate_bound`` (csrc/qce_rate.hip).  ``bussgang_global`` gives the
(B, Cq) pair the scripts build from the global sample covariance for 1 bit and n_bits = inf
(get_Bussgang_matrix / get_Cr, uniform_quantizer.py:60-73, :149-173) from a one-component device model;
the multi-bit Cr of get_Cr uses the quantiser's output variance on its diagonal and is not provided.
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


def bussgang_global(cov, snr, n_bits, device=0):
    """(diag Bussgang gain (N,), Cq = Cr - B C B^H) of Cy = cov + 10^(-snr/10) I (the scripts' Cy_act)."""
    nb = float(n_bits)
    if nb != 1.0 and not np.isinf(nb):
        raise NotImplementedError("multi-bit get_Cr (quantised-variance diagonal) is not provided")
    cov = np.asarray(cov, dtype=complex)
    dm = _lib.DeviceModel(None, cov[None], np.ones(1), device=device)
    try:
        dm.prepare(None, snr, nb)
        t = dm.tables()
    finally:
        dm.close()
    g = np.real(np.diag(t["A_eff"][0]))
    Cq = t["Cr"][0] - (g[:, None] * cov) * g[None, :]
    return g, Cq
