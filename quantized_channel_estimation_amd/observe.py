"""Observations on the device: the scripts' ``get_observation_nbit`` / ``quant`` (reference
modules/utils.py:241-251, :189-203) and the MSE reduction of the estimate loop
(Bussgang_GMM.py:289), computed by libqce.so (``qce_observe`` / ``qce_sq_error``, csrc/qce_observe.hip).

Same names, argument order and output shapes as the reference helpers.  Extra keyword arguments:

* ``noise`` — the CN(0, 1) draw to add (numpy array or CUDA tensor of y's shape).  With it, and
  A = None or a pilot matrix kron(x, I), y is bit-identical to the reference's for the same draw.
* ``seed`` / ``offset`` — without ``noise``, the draw is made on the device by a counter-based
  generator (Philox4x32-10, Box-Muller): complex element e of the batch uses counter offset + e, so
  chunked generation reproduces one-shot generation.  The reference's generator (numpy PCG64,
  unseeded, utils.py:13) cannot be reproduced; its statistics are what the tests check.
* ``device`` — the GPU (default 0).

Host numpy inputs return numpy; ``torch.complex128`` CUDA tensors stay on the device (async on the
current torch stream).
"""
import numpy as np

from . import _lib

_NOISE_NONE, _NOISE_GIVEN, _NOISE_GEN = 0, 1, 2


def _is_tensor(x):
    return not isinstance(x, np.ndarray) and hasattr(x, "data_ptr")


def _nbits(n_bits):
    if n_bits == "inf" or n_bits == np.inf:
        return np.inf
    return float(n_bits)


def _tables(nb, thresholds, quant_labels):
    if nb == 1.0 or np.isinf(nb):
        return None, None, 0
    if thresholds is None or quant_labels is None:
        raise ValueError("multi-bit quantisation needs thresholds and quant_labels")
    thr = np.ascontiguousarray(thresholds, dtype=np.float64).reshape(-1)
    lab = np.ascontiguousarray(quant_labels, dtype=np.float64).reshape(-1)
    if lab.size != thr.size + 1:
        raise ValueError(f"{thr.size} thresholds need {thr.size + 1} labels, got {lab.size}")
    return thr, lab, lab.size


def _stream(t):
    import torch
    return torch.cuda.current_stream(t.device).cuda_stream


def _observe(h2, M, A, scale, noise_kind, w2, seed, offset, nb, thr, lab, nlev, device):
    """h2: (B, N) complex; returns (B, M)."""
    B, N = h2.shape
    a = None if A is None else np.ascontiguousarray(A, dtype=np.complex128)
    if _is_tensor(h2):
        import torch
        if h2.dtype != torch.complex128:
            h2 = h2.to(torch.complex128)
        h2 = h2.contiguous()
        y = torch.empty((B, M), dtype=torch.complex128, device=h2.device)
        if w2 is not None:
            w2 = torch.as_tensor(w2, dtype=torch.complex128, device=h2.device).reshape(B, M).contiguous()
        dev = h2.device.index if h2.device.index is not None else 0
        _lib.check(_lib.load().qce_observe(_lib.ptr(h2), B, N, _lib.ptr(a), M, scale, noise_kind, _lib.ptr(w2),
                                           seed, offset, nb, _lib.ptr(thr), _lib.ptr(lab), nlev, _lib.ptr(y),
                                           dev, _lib.IO_DEVICE, _stream(h2)))
        return y
    h2 = np.ascontiguousarray(h2, dtype=np.complex128)
    if w2 is not None:
        w2 = np.ascontiguousarray(np.asarray(w2, dtype=np.complex128).reshape(B, M))
    y = np.empty((B, M), dtype=np.complex128)
    _lib.check(_lib.load().qce_observe(_lib.ptr(h2), B, N, _lib.ptr(a), M, scale, noise_kind, _lib.ptr(w2), seed,
                                       offset, nb, _lib.ptr(thr), _lib.ptr(lab), nlev, _lib.ptr(y), int(device),
                                       _lib.IO_HOST, None))
    return y


def _squeeze_like_reference(y_full, h_shape):
    """np.squeeze(matmul(A, h[..., None])) then re-insert axis 1 when h.shape[1] == 1 (utils.py:244-246)."""
    if _is_tensor(y_full):
        y = y_full.squeeze()
        if len(h_shape) > 1 and h_shape[1] == 1:
            y = y.unsqueeze(1)
        return y
    y = np.squeeze(y_full)
    if len(h_shape) > 1 and h_shape[1] == 1:
        y = np.expand_dims(y, 1)
    return y


def get_observation_nbit(h, snr, A=None, n_bits=1, thresholds=None, cluster=None, agc=False, *, noise=None,
                         seed=0, offset=0, device=0):
    """y = Q(A h + 10^(-snr/20) n), n ~ CN(0, I) (utils.py:241-251).  ``agc`` is accepted and unused,
    as in the reference."""
    del agc
    nb = _nbits(n_bits)
    thr, lab, nlev = _tables(nb, thresholds, cluster)
    shape = tuple(h.shape)
    N = shape[-1]
    if A is not None and np.asarray(A).shape[1] != N:
        raise ValueError(f"A must have {N} columns")
    M = N if A is None else np.asarray(A).shape[0]
    h2 = h.reshape(-1, N)
    scale = 10 ** (-snr / 20)
    kind = _NOISE_GEN if noise is None else _NOISE_GIVEN
    y = _observe(h2, M, A, scale, kind, noise, int(seed), int(offset), nb, thr, lab, nlev, device)
    return _squeeze_like_reference(y.reshape(*shape[:-1], M), shape)


def quant(inp, n_bits=1, thresholds=None, quant_labels=None, *, device=0):
    """Per-component quantiser (utils.py:189-203) on the device; output has inp's shape."""
    nb = _nbits(n_bits)
    thr, lab, nlev = _tables(nb, thresholds, quant_labels)
    shape = tuple(inp.shape)
    flat = inp.reshape(1, -1) if len(shape) != 2 else inp
    y = _observe(flat, flat.shape[1], None, 0.0, _NOISE_NONE, None, 0, 0, nb, thr, lab, nlev, device)
    return y.reshape(shape)


def sq_error(h_est, h, *, device=0):
    """sum |h_est - h|^2 on the device (deterministic order)."""
    if _is_tensor(h_est):
        import torch
        a = h_est.to(torch.complex128).contiguous()
        b = h.to(torch.complex128).contiguous()
        out = torch.empty(1, dtype=torch.float64, device=a.device)
        dev = a.device.index if a.device.index is not None else 0
        _lib.check(_lib.load().qce_sq_error(_lib.ptr(a), _lib.ptr(b), a.numel(), _lib.ptr(out), dev, _lib.IO_DEVICE,
                                            _stream(a)))
        return out
    a = np.ascontiguousarray(h_est, dtype=np.complex128)
    b = np.ascontiguousarray(h, dtype=np.complex128)
    if a.shape != b.shape:
        raise ValueError("shape mismatch")
    out = np.zeros(1)
    _lib.check(_lib.load().qce_sq_error(_lib.ptr(a), _lib.ptr(b), a.size, _lib.ptr(out), int(device), _lib.IO_HOST,
                                        None))
    return float(out[0])


def mse(h_est, h, *, device=0):
    """The scripts' MSE: sum |h_est - h|^2 / h.size (Bussgang_GMM.py:289)."""
    s = sq_error(h_est, h, device=device)
    n = h.numel() if _is_tensor(h) else np.asarray(h).size
    return s / n
