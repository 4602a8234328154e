"""EM of ``Gmm_quant.fit`` on quantised observations (reference gmm_cplx_quant.py:103-189 fit, :484-602
fit_predict / _initialize_parameters / _initialize, :640-731 _e_step / _m_step, :732-854
estimate_gaussian_parameters / estimate_gaussian_covariances_full, :880-945 estimate_gaussian_covariances_inv;
cov_est_quant.py:31-88 est_cov_from_quant; utils.py:651-700 gauss_newt_solve).

The model of the observations is a GMM with two covariance sets: ``covariances_`` (the recovered
unquantised covariances, what the estimator uses) and ``covariances_quant`` (the covariances of the
quantised data, what the E-step evaluates).  Per iteration the B-sized work runs in libqce.so: the E-step
on ``covariances_quant`` (``qce_em_estep``), the weighted moments nk, means, Q_k = sum r (x-mu)(x-mu)^H / nk
(``qce_em_mstep``, FP64 MFMA), and for multi-bit data two more moment passes over transformed copies of
the observations: the 1-bit signs s = (sign Re d + j sign Im d)/sqrt 2 (Q of s: the arcsine-law
correlation) and the threshold indicators 1(|Re d| < t) + j 1(|Im d| < t) (their weighted means: the
per-dimension probabilities the Gauss-Newton variance fit matches) of d = x (zero-mean models: transformed
once per fit) or d = x - mu_k (models with means: per component and M-step, as the reference's diff at :817),
and the per-component Bussgang gains (the prepare kernels).  The per-component K x (D x D) corrections (sin
law, eigenvalue clipping, the scalar Gauss-Newton solves, the inverse-EM Sigma update of the Toeplitz types,
A Cy A^H with the quantised variances) run on the host in FP64 NumPy, as in the reference.

Covariance types: 'full', 'toeplitz' and 'block-toeplitz' (inverse EM) as the reference.  The reference cannot
complete a fit of 'circulant', 'block-circulant', 'diagonal' or 'spherical' (its M-step helpers for these return
one array where two are unpacked, :758-762) nor of the Toeplitz types at n_bits = inf (est_cov_from_quant reads
absent thresholds); ``reference_fit_error`` reproduces those exceptions (tests/golden/quant_fit_struct.npz).
"""
import warnings

import numpy as np
from scipy.special import erf

from . import _em, _lib
from .rate import quantized_variance


def gauss_newt_solve(f, J, x0, tol=1e-5, maxits=100):
    """utils.py:651-700 (a scalar unknown; the restarts draw from numpy's global RNG as the reference)."""
    dx = 1.0
    xn = x0.copy()
    i = 0
    while (i < maxits) and (np.abs(dx) > tol):
        if np.abs(xn) < 0.1:
            xn = x0 + 0.1 * np.random.randn()
            xn = np.clip(xn, 0.1, 10.0)
        elif np.abs(xn) > 10.0:
            xn = 1.0 + 0.1 * np.random.randn()
        dx = np.linalg.lstsq(np.expand_dims(J(xn), 1), -f(xn), rcond=None)[0][0]
        xn += dx
        i += 1
    return xn, i


def _positive_thresholds(thresholds):
    t = np.asarray(thresholds, dtype=float)
    return t[(t.shape[0] - 1) // 2 + 1:]


def cov_from_quant(corr, probs, nk, thresholds, x0_vec):
    """est_cov_from_quant (cov_est_quant.py:31-88) from its two weighted statistics: corr = sum r s s^H / nk
    of the 1-bit signs and probs (T, 2) = sum r 1(|x_d| < t) / nk (real, imaginary part) per dimension d."""
    D = corr.shape[0]
    corr = np.sin(np.pi / 2 * np.real(corr)) + 1j * np.sin(np.pi / 2 * np.imag(corr))
    thres = _positive_thresholds(thresholds)
    thres = np.concatenate((thres, thres), axis=0)
    s2 = np.zeros(D)
    for d in range(D):
        p = np.clip(probs[d], 1 / nk, (nk - 1) / nk)
        p = np.concatenate((p[:, 0], p[:, 1]), axis=0)

        def f(s, p=p):
            return erf(thres / (np.sqrt(2) * s)) - p

        def jac(s):
            return -np.sqrt(2 / np.pi) * thres * np.exp(-thres ** 2 / (2 * s)) / s ** 2

        x0 = np.real(x0_vec[d])
        v = gauss_newt_solve(f, jac, x0)[0] ** 2
        if np.isnan(v):
            v = 1.0
        s2[d] = np.clip(2 * v, 0, np.inf)
    r = np.sqrt(s2)
    return r[:, None] * corr * r[None, :]


def _eig_clip(c, reg):
    w, Q = np.linalg.eigh(c)
    w = np.clip(w, reg, np.inf)
    return (Q * w) @ Q.conj().T


def quant_covariances(Q, nk, reg, n_bits, sigma2, quantizer, moments, gains):
    """estimate_gaussian_covariances_full (:773-853) from the weighted moments Q_k (K, D, D).
    moments() -> (corr (K, D, D), probs (K, D, T, 2)) for multi-bit data; gains(covs) -> (K, D) Bussgang
    gains of Cy_k = covs_k + sigma2 I.  Returns (covariances, covariances_quant)."""
    K, D, _ = Q.shape
    eye = np.eye(D)
    cov = np.empty_like(Q)
    cq = np.array(Q, copy=True)
    idx = np.arange(D)
    if n_bits == 1:
        for k in range(K):
            c = np.sin(np.pi / 2 * cq[k].real) + 1j * np.sin(np.pi / 2 * cq[k].imag)
            c[idx, idx] += reg
            cq[k][idx, idx] += reg
            w, V = np.linalg.eigh(c)
            w[w < reg] = reg
            c = (V * w) @ V.conj().T
            c[idx, idx] += reg
            cov[k] = c
    elif n_bits != np.inf:
        corr, probs = moments()
        for k in range(K):
            cq[k][idx, idx] += reg
            c = cov_from_quant(corr[k], probs[k], nk[k], quantizer[0], np.diag(cq[k]))
            c = c - sigma2 * eye
            c[idx, idx] += reg
            c = _eig_clip(c, reg)
            c[idx, idx] += reg
            cov[k] = c
        A = gains(cov)
        for k in range(K):
            Cy = cov[k] + sigma2 * eye
            dcr = quantized_variance(np.real(np.diag(Cy)), quantizer[0], quantizer[1])
            c = (A[k][:, None] * Cy) * A[k][None, :].conj()
            c[idx, idx] = dcr
            cq[k] = c
    else:
        for k in range(K):
            c = np.array(cq[k], copy=True)
            c[idx, idx] += reg
            c = c - sigma2 * eye
            c[idx, idx] += reg
            c = _eig_clip(c, reg)
            c[idx, idx] += reg
            cov[k] = c
            cq[k] = c + sigma2 * eye
    return cov, cq


def quant_covariances_inv(Q, nk, reg, n_bits, sigma2, quantizer, moments, gains, F2, Sigma, prev_covs):
    """estimate_gaussian_covariances_inv (:880-945): the recovered covariances of the weighted moments Q_k, then the
    inverse-EM (Barton & Fuhrmann) update of Sigma_k with Cinv = pinv(previous covariances) and
    C_k = F2^H diag(Sigma_k) F2 + reg I.  Sigma (K, P) is updated in place.  Returns (covariances,
    covariances_quant)."""
    K, D, _ = Q.shape
    eye = np.eye(D)
    idx = np.arange(D)
    cov = np.empty_like(Q)
    cq = np.array(Q, copy=True)
    Cinv = np.linalg.pinv(np.asarray(prev_covs), hermitian=True)
    if n_bits == 1:
        for k in range(K):
            c = np.sin(np.pi / 2 * cq[k].real) + 1j * np.sin(np.pi / 2 * cq[k].imag)
            c[idx, idx] += reg
            cq[k][idx, idx] += reg
            w, V = np.linalg.eigh(c)
            w[w < reg] = reg
            cov[k] = (V * w) @ V.conj().T
    else:
        if quantizer is None or quantizer[0] is None:  # est_cov_from_quant reads thresholds.shape (:70)
            raise AttributeError("'NoneType' object has no attribute 'shape'")
        corr, probs = moments()
        for k in range(K):
            cq[k][idx, idx] += reg
            c = cov_from_quant(corr[k], probs[k], nk[k], quantizer[0], np.ones(D))  # x0 = 1 here (no x0_vec)
            c = c - sigma2 * eye
            c[idx, idx] += reg
            cov[k] = _eig_clip(c, reg)
    for k in range(K):
        theta = np.real(F2 @ (Cinv[k] @ cov[k] @ Cinv[k] - Cinv[k]) @ F2.conj().T)
        Sigma[k] = Sigma[k] + Sigma[k] ** 2 * np.diag(theta)
        Sigma[k][Sigma[k] < reg] = reg
        c = (F2.conj().T * Sigma[k]) @ F2
        c[idx, idx] += reg
        cov[k] = c
    if n_bits > 1:
        A = gains(cov)
        for k in range(K):
            Cy = cov[k] + sigma2 * eye
            beta = np.clip(np.real(np.mean(A[k])), 0, 1)
            c = beta ** 2 * Cy
            c[idx, idx] = quantized_variance(np.real(np.diag(Cy)), quantizer[0], quantizer[1])
            cq[k] = c
    return cov, cq


def sigma_init(covs, F2, reg):
    """_initialize's inverse-EM state (:582-586): Sigma_k = Re diag(F2 C_k F2^H), at least reg."""
    S = np.stack([np.real(np.diag(F2 @ c @ F2.conj().T)) for c in covs])
    S[S < reg] = reg
    return S


_UNPACK_TYPES = ("circulant", "block-circulant", "diagonal", "spherical")


def reference_fit_error(covariance_type, n_components, n_bits):
    """The exception the reference's Gmm_quant.fit ends in for a covariance type / bit count it cannot fit (see the
    module docstring), or None.  Pinned to tests/golden/quant_fit_struct.npz."""
    if covariance_type in _UNPACK_TYPES:
        if n_components != 2:
            return ValueError("too many values to unpack (expected 2)")
        if covariance_type == "spherical":
            return np.linalg.LinAlgError("0-dimensional array given. Array must be at least two-dimensional")
        return np.exceptions.AxisError("axis 1 is out of bounds for array of dimension 1")
    if covariance_type in ("toeplitz", "block-toeplitz") and n_bits == np.inf:
        return AttributeError("'NoneType' object has no attribute 'shape'")
    return None


class DeviceBackend:
    """The B-sized work of one fit on the device (data and responsibilities stay resident)."""

    def __init__(self, X, K, reg, zero_mean, n_bits, sigma2, quantizer, quant_type, device):
        self.em = _em.DeviceEM(X, K, "full", reg, zero_mean, device=device)
        self.K, self.device = K, device
        self.n_bits, self.sigma2, self.quantizer, self.quant_type = n_bits, sigma2, quantizer, quant_type
        self.es = self.ez = None
        self.T = 0
        self.X = X
        if n_bits not in (1, np.inf) and quantizer is not None and quantizer[0] is not None:
            self.thr = _positive_thresholds(quantizer[0])
            self.T = self.thr.shape[0]
            if zero_mean:  # d = x for every component: transform once
                S, Z = self._transforms(X)
                self.es = _em.DeviceEM(S, K, "full", 0.0, True, device=device)
                self.ez = _em.DeviceEM(Z, K, "diag", 0.0, False, device=device)

    def _transforms(self, D):
        """1-bit signs of D and the threshold indicators 1(|Re D| < t) + j 1(|Im D| < t), t = the positive
        thresholds (cov_est_quant.py:42-43, :60-63)."""
        S = (np.sign(D.real) + 1j * np.sign(D.imag)) / np.sqrt(2)
        Z = np.concatenate([(np.abs(D.real) < t) + 1j * (np.abs(D.imag) < t) for t in self.thr], axis=1)
        return np.ascontiguousarray(S), np.ascontiguousarray(Z)

    def estep(self, means, covs_quant, weights):
        return self.em.estep(means, covs_quant, weights)

    def mstep(self, resp=None):
        nk, means, cov = self.em.mstep(resp=resp, reg=0.0)
        return nk, means, cov

    def moments(self, resp=None, means=None):
        """(corr (K, D, D), probs (K, D, T, 2)) of d = x (means None) or d = x - mu_k (per component)."""
        R = self.em.R if resp is None else resp
        if means is None:
            _, _, corr = self.es.mstep(resp=R)
            _, pz, _ = self.ez.mstep(resp=R)
        else:
            import torch
            K = self.K
            corr, pz = [], []
            for k in range(K):
                Rk = R[:, k:k + 1].contiguous() if isinstance(R, torch.Tensor) else np.ascontiguousarray(R[:, k:k + 1])
                S, Z = self._transforms(self.X - means[k])
                es = _em.DeviceEM(S, 1, "full", 0.0, True, device=self.device)
                ez = _em.DeviceEM(Z, 1, "diag", 0.0, False, device=self.device)
                try:
                    corr.append(es.mstep(resp=Rk)[2][0])
                    pz.append(ez.mstep(resp=Rk)[1][0])
                finally:
                    es.close()
                    ez.close()
            corr, pz = np.stack(corr), np.stack(pz)
        K, D = corr.shape[0], corr.shape[1]
        pz = pz.reshape(K, self.T, D)  # (K, T, D): real part = Re-indicator mean, imaginary = Im-indicator
        probs = np.stack([np.real(pz), np.imag(pz)], axis=-1).transpose(0, 2, 1, 3)  # (K, D, T, 2)
        return corr, probs

    def gains(self, covs):
        """Bussgang gains of Cy_k = covs_k + sigma2 I (get_Bussgang_matrix of uniform_quantizer.py:60-72 /
        lloyd_max_quantizer.py:10-21) from the prepare kernels (A = I: A_eff = diag gain)."""
        K, D, _ = covs.shape
        dm = _lib.DeviceModel(None, covs, np.full(K, 1.0 / K), device=self.device)
        try:
            kind = _lib.QUANT_LLOYD if self.quant_type == "lloyd" else _lib.QUANT_UNIFORM
            thr = lab = None
            if kind == _lib.QUANT_LLOYD:
                thr, lab = self.quantizer[0], self.quantizer[1]
            dm.prepare(None, -10 * np.log10(self.sigma2), float(self.n_bits), kind, thr, lab)
            A = dm.tables(["A_eff"])["A_eff"]
        finally:
            dm.close()
        return np.real(A[:, np.arange(D), np.arange(D)]).astype(complex)

    def labels(self):
        return self.em.labels()

    def close(self):
        for e in (self.em, self.es, self.ez):
            if e is not None:
                e.close()


def estimate_parameters(obj, be, resp=None, inv=False):
    """estimate_gaussian_parameters (:732-771): nk, means, covariances ('full' branch, or 'inv-em' for the Toeplitz
    types after the initialisation); sets covariances_quant."""
    nk, means, Q = be.mstep(resp)
    centred = None if obj.params.get("zero_mean", False) else means
    moments = lambda: be.moments(resp, centred)  # noqa: E731
    if inv:
        cov, cq = quant_covariances_inv(Q, nk, obj.gm.reg_covar, obj.n_bits, obj.sigma2, obj.quantizer, moments,
                                        be.gains, obj.F2, obj.gm.Sigma, obj.gm.covariances_)
    else:
        cov, cq = quant_covariances(Q, nk, obj.gm.reg_covar, obj.n_bits, obj.sigma2, obj.quantizer, moments,
                                    be.gains)
    obj.covariances_quant = cq
    return nk, means, cov


def fit_predict(obj, X, backend=None):
    """fit_predict (:484-573) with the E-step on covariances_quant and the recovery M-step."""
    gm = obj.gm
    X = np.ascontiguousarray(X, dtype=np.complex128)
    gm.n_features_in_ = X.shape[1]
    if gm.covariance_type != "full":
        raise NotImplementedError(f"Gmm_quant.fit on the device covers covariance_type 'full', not "
                                  f"{gm.covariance_type!r}")
    if getattr(gm, "init_params", "kmeans") not in ("kmeans", "random"):
        raise ValueError("Unimplemented initialization method '%s'" % gm.init_params)
    K = gm.n_components
    zero_mean = bool(obj.params.get("zero_mean", False))
    inv = "inv-em" in obj.params
    if inv and obj.n_bits != 1 and (obj.quantizer is None or obj.quantizer[0] is None):
        raise AttributeError("'NoneType' object has no attribute 'shape'")  # the reference's first M-step
    be = backend or DeviceBackend(X, K, gm.reg_covar, zero_mean, obj.n_bits, obj.sigma2, obj.quantizer,
                                  obj.quant_type, obj.device)
    do_init = not (gm.warm_start and hasattr(obj, "converged_"))
    n_init = gm.n_init if do_init else 1
    max_lower_bound = -np.inf
    gm.converged_ = False
    random_state = _em.check_random_state(gm.random_state)
    n_samples = X.shape[0]
    best_params, best_n_iter, init = None, 0, 0
    try:
        for init in range(n_init):
            if do_init:  # _initialize_parameters / _initialize (:575-638)
                if gm.init_params == "kmeans":
                    from sklearn import cluster
                    resp = np.zeros((n_samples, K))
                    label = cluster.KMeans(n_clusters=K, n_init=1, random_state=random_state).fit(
                        np.concatenate([X.real, X.imag], axis=1)).labels_
                    resp[np.arange(n_samples), label] = 1
                else:
                    resp = random_state.rand(n_samples, K)
                    resp /= resp.sum(axis=1)[:, np.newaxis]
                nk, means, cov = estimate_parameters(obj, be, resp)
                gm.weights_ = nk / n_samples if gm.weights_init is None else gm.weights_init
                gm.means_ = means if gm.means_init is None else gm.means_init
                gm.covariances_ = cov
                if inv:
                    gm.Sigma = sigma_init(cov, obj.F2, gm.reg_covar)
            lower_bound = -np.inf if do_init else gm.lower_bound_
            for n_iter in range(1, gm.max_iter + 1):
                prev_lower_bound = lower_bound
                log_prob_norm = be.estep(gm.means_, obj.covariances_quant, gm.weights_)
                nk, means, cov = estimate_parameters(obj, be, inv=inv)
                gm.weights_, gm.means_, gm.covariances_ = nk / n_samples, means, cov
                lower_bound = log_prob_norm
                print(f"Iteration {n_iter}/{gm.max_iter} | lower bound: {lower_bound}")
                if abs(lower_bound - prev_lower_bound) < gm.tol:
                    gm.converged_ = True
                    break
            if lower_bound > max_lower_bound or best_params is None:
                max_lower_bound = lower_bound
                best_params = (gm.weights_.copy(), gm.means_.copy(), gm.covariances_.copy())
                best_n_iter = n_iter
        if not gm.converged_:
            from sklearn.exceptions import ConvergenceWarning
            warnings.warn("Initialization %d did not converge. Try different init parameters, or increase max_iter, "
                          "tol or check for degenerate data." % (init + 1), ConvergenceWarning)
        gm.weights_, gm.means_, gm.covariances_ = best_params
        gm.n_iter_ = best_n_iter
        gm.lower_bound_ = max_lower_bound
        # the final e-step runs on the last iteration's covariances_quant (:564-566)
        be.estep(gm.means_, obj.covariances_quant, gm.weights_)
        labels = be.labels()
    finally:
        if backend is None:
            be.close()
    gm.precisions_cholesky_ = _em.precision_cholesky(np.asarray(gm.covariances_), device=obj.device) \
        if backend is None else backend.precision_cholesky(np.asarray(gm.covariances_))
    return labels
