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
argmax log r unless every responsibility underflows).  The MFA EM ``fit`` (:94-115, :219-311) is not
provided: adopt a reference-fitted model with ``Mofa.from_reference`` or build one from its factors
with ``Mofa.from_params``.
"""
import numpy as np

from .gmm import Gmm_nbit


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

    def fit(self, data, zero_mean=False):
        raise NotImplementedError("Mofa.fit (MFA EM, mofa_cplx_bussgang.py:94-115) is not provided on the device; "
                                  "adopt a fitted model with Mofa.from_reference or Mofa.from_params")

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
