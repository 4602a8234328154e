"""Drop-in estimate side of the MFA Bussgang estimator ``Mofa`` (reference
modules/mofa_cplx_bussgang.py:10-422).

A mixture of factor analysers is a Gaussian mixture whose covariances are C_k = Lambda_k Lambda_k^H +
diag(psi_k) (``_update_covs`` :313-320; the fitted model keeps them in ``covs``).  Its estimate path
(``estimate_from_y`` :117-160, ``_prepare_for_prediction`` :162-213, ``_lmmse`` :215-216,
``predict_proba`` :342-357) is the Bussgang-GMM path of gmm_cplx_bussgang.py with ``amps`` as the
weights, ``pinvh`` for Cr^-1 and ``slogdet`` for the log-determinant (the same numbers to rounding
for the positive-definite Cr): so it runs on the same libqce.so kernels (dense, Fourier and
large-shape variants) through a ``Gmm_nbit`` core.

Differences kept from the reference: ``estimate_from_y(y, snr_dB, A=None, ...)`` has no
``n_antennas``; A defaults to the identity; mode 1 picks argmax of exp(log r) (:133-136, equal to
argmax log r unless every responsibility underflows).

``fit`` is the reference's MFA EM (:94-115 fit, :219-241 _initialize, :244-265 run_em, :268-320
_EM_per_component / _update_covs, :322-338 _calc_probs, :404-422 _invert_cov_all).  The B-sized work of
every iteration runs on the device: the E-step (log-likelihoods and responsibilities of C_k =
Lambda_k Lambda_k^H + diag psi_k, ``qce_em_estep``) and the responsibility-weighted moments
S0 = sum r, sum r x and sum r (x - m)(x - m)^H (``qce_em_mstep``, FP64 MFMA).  The latents the
reference forms per sample, z_b = beta_k (x_b - mu_k) with beta_k = Lambda_k^H C_k^-1, enter its
M-step only through sums that are linear or quadratic in x, so they follow from those moments:
  sum r z z^H = beta Q(mu, mu) beta^H,   sum r (x - mu') z^H = Q(mu', mu) beta^H,
  sum r (x - Lambda z) = R1 - Lambda beta (R1 - S0 mu),
  sum r ((x - mu') - Lambda z) o conj(x - mu') = diag(Q(mu', mu') - Lambda beta Q(mu, mu')),
with Q(a, c) = sum r (x - a)(x - c)^H.  The per-component K x (D x D) algebra stays on the host, in
FP64 NumPy, as the reference keeps it.  Initialisation is the reference's: sklearn K-means and numpy's
global RNG in the same order, so a seeded global RNG gives the reference's initial parameters.
"""
import numpy as np

from .gmm import Gmm_nbit

EPS10 = 10.0 * np.finfo(np.float64).eps  # qce_em_mstep adds it to nk (sklearn's M-step, gmm :721)


def _update_covs(lambdas, psis):
    """_update_covs (:313-320) with _invert_cov_all (:404-422): C = Lambda Lambda^H + diag psi and its
    Woodbury inverse."""
    K, D, M = lambdas.shape
    lh = np.transpose(lambdas.conj(), (0, 2, 1))
    covs = lambdas @ lh
    covs[:, np.arange(D), np.arange(D)] += psis
    psi_i = 1.0 / psis
    inner = np.linalg.pinv(np.eye(M)[None, :, :] + (lh * psi_i[:, None, :]) @ lambdas)
    step = psi_i[:, :, None] * (lambdas @ inner @ lh) * psi_i[:, None, :]
    for k in range(K):
        step[k] -= np.diag(psi_i[k])
    return covs, -step


def mfa_em(init, stats, maxiter, tol, zero_mean, PPCA=False, lock_psis=False, n_samples=None):
    """run_em (:244-265) over _EM_per_component (:268-311).  init = (means, lambdas, psis, amps);
    stats(means, covs, amps) -> (L, S0, mbar, Qbar, d): the E-step's summed log-likelihood and the
    responsibility-weighted moments S0_k = sum_b r_bk, mbar_k (sum r x / nk, 0 when zero_mean),
    Qbar_k = sum r (x - mbar)(x - mbar)^H and d_k = sum r (x - mbar).  Returns the final parameters,
    covariances, inverse covariances and the lower bound per iteration."""
    means, lambdas, psis, amps = (np.array(a, copy=True) for a in init)
    K, D, M = lambdas.shape
    covs, inv_covs = _update_covs(lambdas, psis)
    L, L_all = -np.inf, []
    eye = np.eye(M)
    i = 0
    for i in range(maxiter):
        newL, S0, mbar, Qbar, d = stats(means, covs, amps)
        betas = np.transpose(lambdas.conj(), (0, 2, 1)) @ inv_covs
        for k in range(K):
            b, s0, mb, dk = betas[k], S0[k], mbar[k], d[k]
            lam, mu = lambdas[k].copy(), means[k].copy()  # the old factors / mean (rows are rewritten below)

            def Q(a, c):
                u, v = mb - a, mb - c
                return Qbar[k] + np.outer(dk, v.conj()) + np.outer(u, dk.conj()) + s0 * np.outer(u, v.conj())

            Qmm = Q(mu, mu)
            lat = s0 * (eye - b @ lam) + b @ Qmm @ b.conj().T
            r1 = dk + s0 * mb
            mu_new = np.zeros(D, complex) if zero_mean else (r1 - lam @ (b @ (r1 - s0 * mu))) / s0
            lambdas[k] = Q(mu_new, mu) @ b.conj().T @ np.linalg.inv(lat)
            ps = np.real(np.diag(Q(mu_new, mu_new) - lam @ b @ Q(mu, mu_new))) / s0
            ps = np.clip(ps, 1e-6, np.inf)
            psis[k] = np.mean(ps) * np.ones(D) if PPCA else ps
            means[k] = mu_new
            amps[k] = s0 / n_samples
        if lock_psis:
            psi = np.dot(S0, psis) / np.sum(S0)
            psis = np.full_like(psis, psi)
        covs, inv_covs = _update_covs(lambdas, psis)
        L_all.append(newL)
        dL = np.abs((newL - L) / newL)
        if i > 5 and dL < tol:
            break
        L = newL
    return means, lambdas, psis, amps, covs, inv_covs, L_all, i


class Mofa:
    def __init__(self, n_components, latent_dim, PPCA=False, lock_psis=False, rs_clip=0.0,
                 max_condition_number=1.e6, maxiter=100, tol=1e-6, verbose=True, device=0):
        self.n_components = n_components
        self.M = latent_dim
        self.PPCA = PPCA
        self.lock_psis = lock_psis
        self.rs_clip = rs_clip
        self.maxiter = maxiter
        self.tol = tol
        self.verbose = verbose
        self.max_condition_number = float(max_condition_number)
        self.device = device
        self.means = self.covs = self.lambdas = self.psis = self.amps = None
        self.inv_covs = None
        self.zero_mean = False
        self.D = None
        self._core = None

    @classmethod
    def from_reference(cls, ref, device=0):
        """Adopt a fitted reference ``Mofa`` (e.g. a joblib-loaded object): reads means, covs, amps,
        lambdas, psis."""
        obj = cls(ref.n_components, ref.M, device=device)
        for name in ("means", "covs", "amps", "lambdas", "psis", "zero_mean", "D"):
            setattr(obj, name, np.copy(getattr(ref, name)) if isinstance(getattr(ref, name, None), np.ndarray)
                    else getattr(ref, name, None))
        obj.amps = np.asarray(obj.amps, dtype=float)
        return obj

    @classmethod
    def from_params(cls, means, lambdas, psis, amps, device=0):
        """C_k = Lambda_k Lambda_k^H + diag(psi_k) (:313-320)."""
        lambdas = np.asarray(lambdas, dtype=complex)
        psis = np.asarray(psis)
        K, D, M = lambdas.shape
        obj = cls(K, M, device=device)
        obj.lambdas, obj.psis = lambdas, psis
        covs = lambdas @ np.transpose(lambdas.conj(), (0, 2, 1))
        covs[:, np.arange(D), np.arange(D)] += psis
        obj.covs = covs
        obj.means = np.zeros((K, D), complex) if means is None else np.asarray(means, complex)
        obj.amps = np.asarray(amps, dtype=float)
        obj.D = D
        return obj

    def _initialize(self, data):
        """_initialize (:219-241): K-means centres (sklearn, numpy's global RNG), random factor loadings,
        per-dimension data variance, random amplitudes -- the reference's draws in its order."""
        from sklearn import cluster
        K, D, M = self.n_components, data.shape[1], self.M
        km = cluster.KMeans(n_clusters=K, n_init=1).fit(np.concatenate([data.real, data.imag], axis=1))
        re, im = np.split(km.cluster_centers_, 2, axis=1)
        means = re + 1j * im
        if self.zero_mean:
            means[:] = 0.0
        lambdas = (np.random.randn(K, D, M) + 1j * np.random.randn(K, D, M)) / np.sqrt(
            self.max_condition_number) / np.sqrt(2)
        psis = np.tile(np.var(data, axis=0)[None, :], (K, 1))
        amps = np.random.rand(K)
        amps /= np.sum(amps)
        return means, lambdas, psis, amps

    def fit(self, data, zero_mean=False, init=None):
        """MFA EM (mofa_cplx_bussgang.py:94-115) with the E-step and the weighted moments on the device
        (module docstring).  init: optional (means, lambdas, psis, amps) in place of _initialize."""
        from . import _em
        data = np.ascontiguousarray(data, dtype=np.complex128)
        self.zero_mean = bool(zero_mean)
        Nd, D = data.shape
        self.N, self.D = Nd, D
        init = self._initialize(data) if init is None else tuple(np.array(a, copy=True) for a in init)
        em = _em.DeviceEM(data, self.n_components, "full", 0.0, self.zero_mean, device=self.device)
        torch = _em._torch()

        def stats(means, covs, amps):
            newL = em.estep(means, covs, amps) * Nd  # _calc_probs: L summed over samples (:322-338)
            if self.rs_clip > 0.0:  # whole components below rs_clip get rs_clip everywhere (:336)
                small = torch.nonzero(em.R.sum(dim=0) < self.rs_clip).flatten()
                if small.numel():
                    em.R[:, small] = self.rs_clip
            nk, mbar, cbar = em.mstep(reg=0.0)
            S0 = nk - EPS10
            return newL, S0, mbar, cbar * nk[:, None, None], (nk - S0)[:, None] * mbar

        try:
            res = mfa_em(init, stats, self.maxiter, self.tol, self.zero_mean, self.PPCA, self.lock_psis, Nd)
        finally:
            em.close()
        self.means, self.lambdas, self.psis, self.amps, self.covs, self.inv_covs, self.L_all, it = res
        if it >= self.maxiter - 1:
            print("\nWarning: EM didn't converge after {0} iterations".format(it))
        elif self.verbose:
            print("EM converged after {0} iterations".format(it))
            print("Final NLL = {0}".format(-self.L_all[-1]))
        self._core = None
        return self

    def __getstate__(self):
        d = self.__dict__.copy()
        d["_core"] = None
        return d

    def __setstate__(self, d):
        self.__dict__.update(d)

    def _gmm(self):
        if self.covs is None:
            raise ValueError("the model has no parameters yet")
        if self._core is None:
            self._core = Gmm_nbit.from_params(self.means, self.covs, self.amps, device=self.device)
        return self._core

    def estimate_from_y(self, y, snr_dB, A=None, n_summands_or_proba=1, n_bits=1, quantizer_type="uniform",
                        quantizer=None):
        """mofa_cplx_bussgang.py:117-160 -> h_est (B, N) in y's dtype."""
        y = np.asarray(y)
        g = self._gmm()
        N = self.covs.shape[-1]
        h = g.estimate_from_y(y, snr_dB, N, A, n_summands_or_proba, n_bits, quantizer_type, quantizer)
        return h.astype(y.dtype, copy=False) if np.iscomplexobj(y) else h

    def predict_proba(self, data):
        """:342-357 (on the model of the last prepare, the channel-domain model before any)."""
        return self._gmm().predict_proba_cplx(np.asarray(data))

    def predict_proba_max(self, data):
        """:359-368."""
        return self._gmm()._predict_cplx(np.asarray(data))
