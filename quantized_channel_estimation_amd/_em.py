"""Device EM for ``Gmm_nbit.fit`` (reference gmm_cplx_bussgang.py:96-163 ``fit``, :437-611
``fit_cplx`` / ``fit_predict`` / ``_initialize_parameters`` / ``_initialize``, :612-697 ``_e_step`` /
``_m_step`` / ``_set_parameters``).

The control flow (n_init restarts, K-means or random initial responsibilities, max_iter / tol
convergence, best lower bound, ConvergenceWarning) mirrors the reference line by line; the
arithmetic of every iteration runs in libqce.so:

* E-step: ``qce_em_estep`` on a device model of the current parameters prepared as the channel-
  domain model (A = I, sigma^2 = 0, no quantisation: Cr = C) -> responsibilities and the lower bound;
* M-step: ``qce_em_mstep`` (FP64 MFMA weighted covariances) -> nk, means, covariances.

Training data and responsibilities stay resident on the device for the whole fit (torch tensors
as plain device buffers).  The K-means initialisation is sklearn's, on the host, as in the
reference (:546-551) — same estimator, same random_state stream, so the same initial labels.
"""
import warnings

import numpy as np

from . import _lib


def _torch():
    import torch
    return torch


def check_random_state(seed):
    """sklearn.utils.check_random_state semantics (the reference's ut.check_random_state, utils.py:593)."""
    from sklearn.utils import check_random_state as _crs
    return _crs(seed)


class DeviceEM:
    """EM state of one fit: X (B, N) complex128 on ``device``; parameters on the host (small)."""

    def __init__(self, X, n_components, covariance_type, reg_covar, zero_mean, device=0):
        torch = _torch()
        self.device = int(device)
        self.dev = torch.device("cuda", self.device)
        X = np.ascontiguousarray(X, dtype=np.complex128)
        if X.ndim != 2:
            raise ValueError("X must be (n_samples, n_features)")
        self.B, self.N = X.shape
        self.K = int(n_components)
        if self.N > 256:
            raise NotImplementedError("device EM supports n_features <= 256")
        self.diag = covariance_type == "diag"
        if covariance_type not in ("full", "diag"):
            raise NotImplementedError(f"device EM supports 'full' and 'diag' covariances, not {covariance_type!r}")
        self.reg = float(reg_covar)
        self.zero_mean = bool(zero_mean)
        self.X = torch.from_numpy(X).to(self.dev)
        self.R = torch.empty((self.B, self.K), dtype=torch.float64, device=self.dev)
        self.lse = torch.empty(1, dtype=torch.float64, device=self.dev)
        self.nk = torch.empty(self.K, dtype=torch.float64, device=self.dev)
        self.mu = torch.empty((self.K, self.N), dtype=torch.complex128, device=self.dev)
        shape = (self.K, self.N) if self.diag else (self.K, self.N, self.N)
        self.cov = torch.empty(shape, dtype=torch.float64 if self.diag else torch.complex128, device=self.dev)
        self._dm = None

    def _stream(self):
        return _torch().cuda.current_stream(self.dev).cuda_stream

    def mstep(self, resp=None, reg=None):
        """estimate_gaussian_parameters (:698-737) on the device; resp None = the last E-step's."""
        torch = _torch()
        reg = self.reg if reg is None else float(reg)
        if resp is None:
            R = self.R
        elif isinstance(resp, torch.Tensor):  # device responsibilities of another DeviceEM on this GPU
            R = resp.contiguous()
        else:
            R = torch.as_tensor(np.ascontiguousarray(resp, dtype=np.float64), device=self.dev)
        _lib.check(_lib.load().qce_em_mstep(_lib.ptr(self.X), self.B, self.N, self.K, _lib.ptr(R), reg,
                                            int(self.diag), int(self.zero_mean), _lib.ptr(self.nk),
                                            _lib.ptr(self.mu), _lib.ptr(self.cov), self.device, _lib.IO_DEVICE,
                                            self._stream()))
        nk = self.nk.cpu().numpy()
        means = self.mu.cpu().numpy()
        cov = self.cov.cpu().numpy()
        return nk, means, cov

    def estep(self, means, covs_full, weights):
        """_e_step (:612-630): responsibilities into self.R, returns mean log p(x)."""
        _torch().cuda.current_stream(self.dev).synchronize()  # R / X consumers done before tables change
        if self._dm is None:
            self._dm = _lib.DeviceModel(means, covs_full, weights, device=self.device)
        else:
            self._dm.set_params(means, covs_full, weights)
        self._dm.prepare(None, float("inf"), float("inf"), stream=self._stream())
        _lib.check(_lib.load().qce_em_estep(self._dm.handle, _lib.ptr(self.X), self.B, _lib.ptr(self.R),
                                            _lib.ptr(self.lse), _lib.IO_DEVICE, self._stream()))
        # torch's default stream has handle 0, which the model-bound entry points read as "the model's own
        # (non-blocking) stream": finish that stream before torch-side reads of R / lse
        self._dm.synchronize()
        return float(self.lse.cpu().numpy()[0])

    def close(self):
        if self._dm is not None:
            _torch().cuda.current_stream(self.dev).synchronize()
            self._dm.close()
            self._dm = None

    def toeplitz_step(self, S, F2, sigma, init):
        """Inverse-EM covariance step (:792-826); init: the Sigma of _initialize (:582-586).
        Returns (sigma, covariances or None)."""
        S = np.ascontiguousarray(S, dtype=np.complex128)
        F2 = np.ascontiguousarray(F2, dtype=np.complex128)
        sigma = np.ascontiguousarray(sigma, dtype=np.float64).copy()
        covs = None if init else np.empty((self.K, self.N, self.N), dtype=np.complex128)
        _torch().cuda.current_stream(self.dev).synchronize()
        h = None if init else self._dm.handle
        _lib.check(_lib.load().qce_em_toeplitz(h, _lib.ptr(S), self.K, self.N, _lib.ptr(F2), F2.shape[0],
                                               _lib.ptr(sigma), self.reg, int(init), _lib.ptr(covs), self.device,
                                               None if init else self._stream()))
        return sigma, covs

    def labels(self):
        return self.R.argmax(dim=1).cpu().numpy()


def full_of(cov, diag):
    """Dense (K, N, N) complex covariances of 'full' or 'diag' parameters."""
    if not diag:
        return np.asarray(cov, dtype=complex)
    K, N = cov.shape
    out = np.zeros((K, N, N), dtype=complex)
    out[:, np.arange(N), np.arange(N)] = cov
    return out


def precision_cholesky(covs_full, device=0):
    """compute_precision_cholesky(covs, 'full') (:15-52) via the device prepare: P_k = (L_k^-1)^H."""
    dm = _lib.DeviceModel(None, covs_full, np.full(covs_full.shape[0], 1.0 / covs_full.shape[0]), device=device)
    try:
        dm.prepare(None, float("inf"), float("inf"))
        return dm.tables()["P"]
    finally:
        dm.close()


def fit_predict(obj, X):
    """The reference's fit_predict (:462-536) for the device; ``obj`` is a Gmm_nbit."""
    gm = obj.gm
    X = np.asarray(X)
    gm.n_features_in_ = X.shape[1]  # _check_n_features(X, reset=True) (:487)
    if getattr(gm, "init_params", "kmeans") not in ("kmeans", "random"):
        raise ValueError("Unimplemented initialization method '%s'" % gm.init_params)
    if getattr(gm, "precisions_init", None) is not None:
        raise NotImplementedError("precisions_init is not supported by the device EM")
    inv_em = "inv-em" in obj.params
    K = gm.n_components
    do_init = not (gm.warm_start and hasattr(obj, "converged_"))  # the reference tests the wrapper (:491)
    n_init = gm.n_init if do_init else 1
    max_lower_bound = -np.inf
    gm.converged_ = False
    random_state = check_random_state(gm.random_state)
    em = DeviceEM(X, K, gm.covariance_type, gm.reg_covar, obj.params.get("zero_mean", False), device=obj.device)
    n_samples = X.shape[0]
    best_params, best_n_iter = None, 0
    lower_bound, n_iter = -np.inf, 0
    for init in range(n_init):
        if do_init:
            _initialize_parameters(obj, em, X, random_state)
        lower_bound = -np.inf if do_init else gm.lower_bound_
        for n_iter in range(1, gm.max_iter + 1):
            prev_lower_bound = lower_bound
            log_prob_norm = em.estep(gm.means_, full_of(gm.covariances_, em.diag), gm.weights_)
            if inv_em:  # estimate_gaussian_covariances_inv (:792-826)
                nk, means, S = em.mstep(reg=0.0)
                gm.Sigma, cov = em.toeplitz_step(S, obj.F2, gm.Sigma, init=False)
            else:
                nk, means, cov = em.mstep()
            gm.weights_, gm.means_, gm.covariances_ = nk / n_samples, means, cov
            lower_bound = log_prob_norm
            change = lower_bound - prev_lower_bound
            if abs(change) < gm.tol:
                gm.converged_ = True
                break
        if lower_bound > max_lower_bound or best_params is None:
            max_lower_bound = lower_bound
            best_params = (gm.weights_.copy(), gm.means_.copy(), gm.covariances_.copy())
            best_n_iter = n_iter
    if not gm.converged_:
        from sklearn.exceptions import ConvergenceWarning
        warnings.warn("Initialization %d did not converge. Try different init parameters, or increase max_iter, tol "
                      "or check for degenerate data." % (init + 1), ConvergenceWarning)
    gm.weights_, gm.means_, gm.covariances_ = best_params
    covs_full = full_of(gm.covariances_, em.diag)
    if em.diag:
        gm.precisions_cholesky_ = 1.0 / np.sqrt(gm.covariances_)
        gm.precisions_ = np.abs(gm.precisions_cholesky_) ** 2
    else:
        P = precision_cholesky(covs_full, device=obj.device)
        gm.precisions_cholesky_ = P
        gm.precisions_ = np.einsum("kij,klj->kil", P, P.conj())
    gm.n_iter_ = best_n_iter
    gm.lower_bound_ = max_lower_bound
    em.estep(gm.means_, covs_full, gm.weights_)  # final e-step (:532-534)
    labels = em.labels()
    em.close()
    return labels


def _initialize_parameters(obj, em, X, random_state):
    """:538-556 then _initialize (:558-590)."""
    gm = obj.gm
    n_samples = X.shape[0]
    if gm.init_params == "kmeans":
        from sklearn import cluster
        resp = np.zeros((n_samples, gm.n_components))
        X_real = np.concatenate([X.real, X.imag], axis=1)  # ut.cplx2real(X, axis=1), utils.py:504-508
        label = cluster.KMeans(n_clusters=gm.n_components, n_init=1, random_state=random_state).fit(X_real).labels_
        resp[np.arange(n_samples), label] = 1
    else:
        resp = random_state.rand(n_samples, gm.n_components)
        resp /= resp.sum(axis=1)[:, np.newaxis]
    nk, means, cov = em.mstep(resp)
    weights = nk / n_samples
    gm.weights_ = weights if gm.weights_init is None else gm.weights_init
    gm.means_ = means if gm.means_init is None else gm.means_init
    gm.covariances_ = cov
    if "inv-em" in obj.params:  # :582-586
        gm.Sigma, _ = em.toeplitz_step(cov, obj.F2, np.zeros((gm.n_components, obj.F2.shape[0])), init=True)
