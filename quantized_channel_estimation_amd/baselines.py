"""Global and genie Bussgang-LMMSE baselines on the device (reference estimators/blmmse.py:6-97,
called by Bussgang_GMM.py:102-165 through ``mp_eval``).

* ``estimate_global(y, C, ...)``: one covariance for every sample = a one-component, zero-mean
  mixture; its 'all'-mode estimate is exactly h = C A_eff^H Cr^-1 y (the responsibility of the only
  component is 1).
* ``estimate_genie(y, t, ...)``: sample b has its own covariance C_b = toeplitz(t_b)^T (:27, :44, :51):
  a mixture with one component per sample, prepared in one batched FP64 pass (the per-component
  Cholesky / Bussgang / filter kernels of the estimate path), then h_b = W_b y_b
  (``qce_estimate_assigned``).  Processed in chunks of samples to bound device memory.

The reference mixes the multi-bit Cr with the first Bussgang gain (:53, :86); the models here are
created with ``QCE_OPT_BETA_FIRST`` so the arithmetic is the same.  A custom ``Cr`` (:64, :90) is not
supported.
"""
import numpy as np

from . import _lib
from .gmm import _nbits_of


def _qparams(n_bits, quantizer_type, quantizer):
    nb = _nbits_of(n_bits)
    if nb == 1 or np.isinf(nb):
        return nb, _lib.QUANT_UNIFORM, None, None
    if quantizer_type == "uniform":
        return nb, _lib.QUANT_UNIFORM, None, None
    if quantizer_type == "lloyd":
        return nb, _lib.QUANT_LLOYD, np.asarray(quantizer[0], float), np.asarray(quantizer[1], float)
    # the reference leaves A_buss = None and fails in A_buss @ A (:57-58)
    raise TypeError("unsupported operand type(s) for @: 'NoneType' and 'numpy.ndarray'")


def _toeplitz_covs(t):
    """C_b = toeplitz(t_b)^T for every row of t (modules/utils.py:115 toeplitz with r = conj(c))."""
    t = np.asarray(t, dtype=complex)
    N = t.shape[-1]
    i = np.arange(N)
    d = i[None, :] - i[:, None]  # j - i
    T = np.where(d[None] >= 0, np.conj(t)[:, np.abs(d)], t[:, np.abs(d)])  # toeplitz(c): [i][j] = c[i-j] or conj
    return np.ascontiguousarray(np.transpose(T, (0, 2, 1)))


class BLMMSE:
    def __init__(self, snr, device=0, chunk=4096):
        self.snr = snr
        self.rho = 10 ** (0.1 * snr)
        self.sigma2 = 1 / self.rho
        self.device = device
        self.chunk = int(chunk)

    def __getstate__(self):
        return self.__dict__.copy()

    def _model(self, covs, A, n_bits, quantizer_type, quantizer):
        nb, qk, thr, lab = _qparams(n_bits, quantizer_type, quantizer)
        K = covs.shape[0]
        dm = _lib.DeviceModel(None, covs, np.full(K, 1.0 / K), device=self.device)
        dm.set_option(_lib.OPT_BETA_FIRST, 1)
        a = None if A is None else np.asarray(A, dtype=complex)
        dm.prepare(a, self.snr, nb, qk, thr, lab)
        return dm

    def estimate_global(self, y, C, A=None, n_bits=1, quantizer_type="uniform", quantizer=None, Cr=None):
        """blmmse.py:64-97."""
        if Cr is not None:
            raise NotImplementedError("a user-supplied Cr is not supported")
        y = np.asarray(y)
        dm = self._model(np.asarray(C, dtype=complex)[None], A, n_bits, quantizer_type, quantizer)
        try:
            h = dm.estimate(np.ascontiguousarray(y, dtype=np.complex128), _lib.MODE_ALL, 0.0)
        finally:
            dm.close()
        return h.astype(y.dtype, copy=False) if np.iscomplexobj(y) else h

    def estimate_genie(self, y, t, A=None, n_bits=1, quantizer_type="uniform", quantizer=None, Cr=None):
        """blmmse.py:20-62: per-sample covariance toeplitz(t_b)^T."""
        if Cr is not None:
            raise NotImplementedError("a user-supplied Cr is not supported")
        y = np.asarray(y)
        t = np.asarray(t)
        B = y.shape[0]
        N = t.shape[-1]
        out = np.empty((B, N), dtype=np.complex128)
        for s in range(0, B, self.chunk):
            e = min(B, s + self.chunk)
            dm = self._model(_toeplitz_covs(t[s:e]), A, n_bits, quantizer_type, quantizer)
            try:
                out[s:e] = dm.estimate_assigned(y[s:e])
            finally:
                dm.close()
        return out.astype(y.dtype, copy=False) if np.iscomplexobj(y) else out


def _ls_kind(A):
    """True for column-orthogonal A (I or kron(x, I): the per-column kernel), "general" for any other A with
    at least as many rows as columns (device pseudo-inverse)."""
    if A is None:
        return True
    A = np.asarray(A, dtype=complex)
    G = A.conj().T @ A
    if np.abs(G - np.diag(np.diag(G))).max() <= 1e-12 * np.abs(np.diag(G)).max():
        return True
    if A.shape[0] < A.shape[1]:
        raise NotImplementedError("LS on the device needs column-orthogonal A or A with M >= N")
    return "general"


class LS:
    """Bussgang least squares (estimators/LS.py:15-76): h = lstsq(A_eff, y), A_eff = G A with the Bussgang
    gain G of the global (estimate_global) or per-sample (estimate_genie) covariance."""

    def __init__(self, snr, device=0, chunk=4096):
        self.snr = snr
        self.rho = 10 ** (0.1 * snr)
        self.sigma2 = 1 / self.rho
        self.device = device
        self.chunk = int(chunk)

    def _run(self, y, covs, A, n_bits, quantizer_type, quantizer, per_sample):
        kind = _ls_kind(A)
        y = np.asarray(y)
        est = BLMMSE(self.snr, device=self.device)
        B = y.shape[0]
        N = covs.shape[-1]
        out = np.empty((B, N), dtype=np.complex128)
        step = self.chunk if per_sample else max(B, 1)
        for s in range(0, B, step):
            e = min(B, s + step)
            dm = est._model(covs[s:e] if per_sample else covs, A, n_bits, quantizer_type, quantizer)
            try:
                comp = None if per_sample else np.zeros(e - s, dtype=np.int64)
                out[s:e] = dm.estimate_assigned(y[s:e], comp, ls=kind)
            finally:
                dm.close()
        return out

    def estimate_global(self, y, C, A=None, n_bits=1, quantizer_type="uniform", quantizer=None):
        """LS.py:55-76."""
        y = np.asarray(y)
        h = self._run(y, np.asarray(C, dtype=complex)[None], A, n_bits, quantizer_type, quantizer, False)
        return h.astype(y.dtype, copy=False) if np.iscomplexobj(y) else h

    def estimate_genie(self, y, t, A=None, n_bits=1, quantizer_type="uniform", quantizer=None):
        """LS.py:21-53 (NaN rows -> 0, :48-52)."""
        if n_bits == "inf" or n_bits == np.inf:
            # LS.py:35-37 assigns lstsq's result tuple to a row, which numpy rejects
            raise ValueError("setting an array element with a sequence.")
        y = np.asarray(y)
        h = self._run(y, _toeplitz_covs(t), A, n_bits, quantizer_type, quantizer, True)
        h[np.isnan(h).any(axis=1)] = 0
        return h.astype(y.dtype, copy=False) if np.iscomplexobj(y) else h


def mp_LS_global(obj, *args):
    """Bussgang_GMM.py:25-26."""
    return obj.estimate_global(*args)


def mp_LS_genie(obj, *args):
    """Bussgang_GMM.py:22-23."""
    return obj.estimate_genie(*args)


def mp_eval(obj, y, toep, h_true, genie, A=None, n_bits=1, quantizer_type=None, quantizer=None, Cr=None):
    """blmmse.py:7-12 (the scripts' pool worker)."""
    if genie:
        return obj.estimate_genie(y, toep, A, n_bits, quantizer_type, quantizer, Cr)
    return obj.estimate_global(y, toep, A, n_bits, quantizer_type, quantizer, Cr)
