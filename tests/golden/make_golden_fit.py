"""Generate tests/golden/fit.npz: golden vectors for the device EM fit (SURVEY.md §8(f) 1;
reference gmm_cplx_bussgang.py:96-163 `fit`, :437-790 EM).

Runs ONLY in the build container, where /root/reference exists (imported read-only, no bytecode
written, the same three harness-side API-drift shims as make_golden.py).  For each case it stores
the training channels, the hyper-parameters, and the reference's fitted means_cplx, covs_cplx,
gm.weights_, gm.n_iter_, gm.lower_bound_, gm.converged_, and for the Fourier fits fft_means /
fft_covs.  Also one K-means-initialised responsibility matrix and the reference's M-step on it
(estimate_gaussian_parameters) as a single-step known answer.

Usage:  python -B tests/golden/make_golden_fit.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def main():
    import warnings
    import numpy as np
    from make_golden import _import_reference
    R = _import_reference()
    gmm_mod = R["gmm"]
    warnings.simplefilter("ignore")
    out = {}
    scm = R["SCMMulti"](path_sigma=2.0, n_path=1)
    h16, _ = scm.generate_channel(1200, 1, 16, np.random.default_rng(4321))
    h16 = np.squeeze(h16).astype(complex)
    out["h16"] = h16
    cases = [
        ("full_zm", "full", None, True, dict(n_components=6, random_state=0, max_iter=12)),
        ("full_mean", "full", None, False, dict(n_components=6, random_state=1, max_iter=12)),
        ("full_rand", "full", None, True, dict(n_components=4, random_state=2, max_iter=8, init_params="random")),
        ("circ", "circulant", None, True, dict(n_components=6, random_state=0, max_iter=12)),
        ("bcirc", "block-circulant", (2, 8), False, dict(n_components=5, random_state=3, max_iter=12)),
        ("full_ninit", "full", None, True, dict(n_components=4, random_state=5, max_iter=6, n_init=2)),
        ("toep", "toeplitz", None, True, dict(n_components=5, random_state=0, max_iter=10)),
        ("btoep", "block-toeplitz", (2, 8), False, dict(n_components=4, random_state=4, max_iter=8)),
    ]
    tags = []
    from threadpoolctl import threadpool_limits
    for tag, ct, blocks, zm, kw in cases:
        g = gmm_mod.Gmm_nbit(covariance_type=ct, **kw)
        # sklearn's threaded K-means adds per-thread partial centres in completion order, so its
        # labels (and the whole EM trajectory after them) can change from run to run: one thread here
        # and in the test keeps the initialisation reproducible.
        with threadpool_limits(limits=1):
            g.fit(h16, blocks=blocks, zero_mean=zm)
        p = tag + "__"
        out[p + "cov_type"] = np.array(ct)
        out[p + "blocks"] = np.array(blocks if blocks else (0, 0))
        out[p + "zero_mean"] = np.bool_(zm)
        for k, v in kw.items():
            out[p + "kw_" + k] = np.array(v)
        out[p + "means_cplx"] = np.asarray(g.means_cplx)
        out[p + "covs_cplx"] = np.asarray(g.covs_cplx)
        out[p + "weights"] = np.asarray(g.gm.weights_)
        out[p + "n_iter"] = np.int64(g.gm.n_iter_)
        out[p + "lower_bound"] = np.float64(g.gm.lower_bound_)
        out[p + "converged"] = np.bool_(g.gm.converged_)
        out[p + "chol"] = np.asarray(g.chol)
        if getattr(g.gm, "Sigma", None) is not None:
            out[p + "Sigma"] = np.asarray(g.gm.Sigma)
        if g.fft_covs is not None:
            out[p + "fft_covs"] = np.asarray(g.fft_covs)
            out[p + "fft_means"] = np.asarray(g.fft_means)
        tags.append(tag)
    out["tags"] = np.array(tags)
    # single M-step known answer on a fixed responsibility matrix ('full' and 'diag')
    rng = np.random.default_rng(11)
    resp = rng.random((h16.shape[0], 5))
    resp /= resp.sum(axis=1, keepdims=True)
    g = gmm_mod.Gmm_nbit(n_components=5, covariance_type="full", reg_covar=1e-6)
    g.params["zero_mean"] = False
    nk, mu, cov = g.estimate_gaussian_parameters(h16, resp, 1e-6, "full")
    _, _, covd = g.estimate_gaussian_parameters(h16, resp, 1e-6, "diag")
    g.params["zero_mean"] = True
    _, mu0, cov0 = g.estimate_gaussian_parameters(h16, resp, 1e-6, "full")
    out.update(mstep_resp=resp, mstep_nk=nk, mstep_means=mu, mstep_covs=cov, mstep_diag=covd, mstep_covs_zm=cov0,
               mstep_means_zm=mu0)
    np.savez_compressed(os.path.join(HERE, "fit.npz"), **out)
    print("wrote fit.npz:", tags)


if __name__ == "__main__":
    main()
