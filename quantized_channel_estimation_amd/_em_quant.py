"""EM of ``Gmm_quant.fit`` on quantised observations, 'full' covariances (reference gmm_cplx_quant.py:103-189
fit, :484-602 fit_predict / _initialize_parameters / _initialize, :640-731 _e_step / _m_step,
:732-854 estimate_gaussian_parameters / estimate_gaussian_covariances_full; cov_est_quant.py:31-88
est_cov_from_quant; utils.py:651-700 gauss_newt_solve).

The model of the observations is a GMM with two covariance sets: ``covariances_`` (the recovered
unquantised covariances, what the estimator uses) and ``covariances_quant`` (the covariances of the
quantised data, what the E-step evaluates).  Per iteration the B-sized work runs in libqce.so: the E-step
on ``covariances_quant`` (``qce_em_estep``), the weighted moments nk, means, Q_k = sum r (x-mu)(x-mu)^H / nk
(``qce_em_mstep``, FP64 MFMA), and for multi-bit data two more moment passes over transformed copies of
the observations: the 1-bit signs s = (sign Re x + j sign Im x)/sqrt 2 (Q of s: the arcsine-law
correlation) and the threshold indicators 1(|Re x| < t) + j 1(|Im x| < t) (their weighted means: the
per-dimension probabilities the Gauss-Newton variance fit matches), and the per-component Bussgang gains
(the prepare kernels).  The per-component K x (D x D) corrections (sin law, eigenvalue clipping, the
scalar Gauss-Newton solves, A Cy A^H with the quantised variances) run on the host in FP64 NumPy, as in
the reference.  Multi-bit data with non-zero means would need per-component sign / indicator transforms
of x - mu_k and raises NotImplementedError (the reference script fits zero-mean models,
Bussgang_GMM_quant.py:47).
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


class DeviceBackend:
    """The B-sized work of one fit on the device (data and responsibilities stay resident)."""

    def __init__(self, X, K, reg, zero_mean, n_bits, sigma2, quantizer, quant_type, device):
        self.em = _em.DeviceEM(X, K, "full", reg, zero_mean, device=device)
        self.K, self.device = K, device
        self.n_bits, self.sigma2, self.quantizer, self.quant_type = n_bits, sigma2, quantizer, quant_type
        self.es = self.ez = None
        self.T = 0
        if n_bits not in (1, np.inf):
            if not zero_mean:
                raise NotImplementedError("Gmm_quant.fit: multi-bit covariance recovery with non-zero means "
                                          "(per-component sign / threshold transforms of x - mu_k) is not provided")
            S = (np.sign(X.real) + 1j * np.sign(X.imag)) / np.sqrt(2)
            thr = _positive_thresholds(quantizer[0])
            self.T = thr.shape[0]
            Z = np.concatenate([(np.abs(X.real) < t) + 1j * (np.abs(X.imag) < t) for t in thr], axis=1)
            self.es = _em.DeviceEM(S, K, "full", 0.0, True, device=device)
            self.ez = _em.DeviceEM(np.ascontiguousarray(Z), K, "diag", 0.0, False, device=device)

    def estep(self, means, covs_quant, weights):
        return self.em.estep(means, covs_quant, weights)

    def mstep(self, resp=None):
        nk, means, cov = self.em.mstep(resp=resp, reg=0.0)
        return nk, means, cov

    def moments(self, resp=None):
        R = self.em.R if resp is None else resp
        _, _, corr = self.es.mstep(resp=R)
        _, pz, _ = self.ez.mstep(resp=R)
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


def estimate_parameters(obj, be, resp=None):
    """estimate_gaussian_parameters (:732-771) for 'full': nk, means, covariances; sets covariances_quant."""
    nk, means, Q = be.mstep(resp)
    cov, cq = quant_covariances(Q, nk, obj.gm.reg_covar, obj.n_bits, obj.sigma2, obj.quantizer,
                                lambda: be.moments(resp), be.gains)
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
            lower_bound = -np.inf if do_init else gm.lower_bound_
            for n_iter in range(1, gm.max_iter + 1):
                prev_lower_bound = lower_bound
                log_prob_norm = be.estep(gm.means_, obj.covariances_quant, gm.weights_)
                nk, means, cov = estimate_parameters(obj, be)
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
