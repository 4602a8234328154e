"""Generate tests/golden/quant_fit_struct.npz: the reference's Gmm_quant.fit beyond the zero-mean 'full' cases of
quant_fit.npz --

  * 'toeplitz' / 'block-toeplitz': the inverse-EM M-step on quantised data (gmm_cplx_quant.py:166-181 fit,
    :582-586 the Sigma initialisation, :880-945 estimate_gaussian_covariances_inv), 1 / 2 / 3 bits, zero mean
    and with means;
  * 'full' multi-bit with means (est_cov_from_quant on x - mu_k, :817);
  * the covariance types whose fit the reference cannot complete -- 'circulant', 'block-circulant', 'diagonal',
    'spherical' (their M-step helpers return one array where two are unpacked, :758-762) and 'toeplitz' at
    n_bits = inf (est_cov_from_quant reads the absent thresholds): the exception type and message.

Runs ONLY in the build container (reference imported read-only through make_golden.py's harness).  Data and
seeding as make_golden_quant_fit.py: SCM channels, the reference's own quant on seeded noise, one k-means
thread, numpy's global RNG seeded before each fit (Gauss-Newton restarts).

Usage:  python -B tests/golden/make_golden_quant_fit_struct.py
"""
import contextlib
import io
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

CASES = [  # tag, covariance type, blocks, n_bits, quantizer type, zero_mean, K, max_iter, snr
    ("t_b1_zm", "toeplitz", None, 1, "uniform", True, 3, 6, 5.0),
    ("t_b2u_zm", "toeplitz", None, 2, "uniform", True, 3, 5, 5.0),
    ("t_b3l_mean", "toeplitz", None, 3, "lloyd", False, 2, 5, 10.0),
    ("bt_b1_mean", "block-toeplitz", (2, 4), 1, "uniform", False, 3, 5, 0.0),
    ("bt_b2u_zm", "block-toeplitz", (2, 4), 2, "uniform", True, 2, 5, 5.0),
    ("f_b2u_mean", "full", None, 2, "uniform", False, 2, 5, 5.0),
    ("f_b3l_mean", "full", None, 3, "lloyd", False, 3, 4, 10.0),
]
ERRORS = [  # tag, covariance type, blocks, n_bits, quantizer type, K
    ("e_circ3", "circulant", None, 1, "uniform", 3),
    ("e_circ2", "circulant", None, 2, "uniform", 2),
    ("e_bcirc3", "block-circulant", (2, 4), 2, "uniform", 3),
    ("e_bcirc2", "block-circulant", (2, 4), 1, "uniform", 2),
    ("e_diag3", "diagonal", None, 1, "uniform", 3),
    ("e_diag2", "diagonal", None, 2, "uniform", 2),
    ("e_sph3", "spherical", None, 1, "uniform", 3),
    ("e_sph2", "spherical", None, 1, "uniform", 2),
    ("e_tinf", "toeplitz", None, "inf", "uniform", 3),
    ("e_btinf", "block-toeplitz", (2, 4), "inf", "uniform", 2),
]


def main():
    import warnings
    import numpy as np
    from threadpoolctl import threadpool_limits
    from make_golden import _import_reference
    R = _import_reference()
    ut = R["ut"]
    Gmm_quant = R["gmmq"].Gmm_quant
    warnings.simplefilter("ignore")
    scm = R["SCMMulti"](path_sigma=2.0, n_path=2)
    h, _ = scm.generate_channel(1200, 1, 8, np.random.default_rng(15))
    h = np.squeeze(h).astype(complex)
    out = dict(h=h)
    rng = np.random.default_rng(16)

    def observe(n_bits, qt, snr):
        quantizer = ut.get_quantizer([snr], n_bits, qt)[snr] if n_bits not in (1, np.inf) else (None, None, None)
        w = (rng.standard_normal(h.shape) + 1j * rng.standard_normal(h.shape)) * np.sqrt(0.5)
        y = h + 10 ** (-snr / 20) * w
        if n_bits != np.inf:
            y = ut.quant(y, n_bits, quantizer[0], quantizer[1])
        return y, quantizer

    tags = []
    for tag, ct, blocks, nb, qt, zm, K, max_iter, snr in CASES:
        y, quantizer = observe(nb, qt, snr)
        sigma2 = 10 ** (-snr / 10)
        g = Gmm_quant(n_components=K, covariance_type=ct, max_iter=max_iter, random_state=0)
        np.random.seed(123)
        with threadpool_limits(limits=1), contextlib.redirect_stdout(io.StringIO()):
            g.fit(h=y, n_bits=nb, sigma2=sigma2, quantizer=quantizer, quant_type=qt, blocks=blocks, zero_mean=zm)
        p = tag + "__"
        out[p + "y"] = y
        out[p + "cfg"] = np.array([float(nb), float(zm), K, max_iter, snr, sigma2])
        out[p + "ctype"] = np.array(ct)
        out[p + "blocks"] = np.array(blocks if blocks else (0, 0))
        out[p + "qtype"] = np.array(qt)
        if quantizer[0] is not None:
            out[p + "thr"], out[p + "lab"] = np.asarray(quantizer[0]), np.asarray(quantizer[1])
        out[p + "weights"] = g.gm.weights_
        out[p + "means"] = g.means_cplx
        out[p + "covs"] = g.covs_cplx
        out[p + "chol"] = g.chol
        out[p + "covs_quant"] = g.covariances_quant
        out[p + "n_iter"] = np.int64(g.gm.n_iter_)
        out[p + "lower_bound"] = np.float64(g.gm.lower_bound_)
        out[p + "converged"] = np.bool_(g.gm.converged_)
        if "inv-em" in g.params:
            out[p + "Sigma"] = g.gm.Sigma
            out[p + "F2"] = g.F2
        tags.append(tag)
    etags = []
    for tag, ct, blocks, nb, qt, K in ERRORS:
        n_bits = np.inf if nb == "inf" else nb
        y, quantizer = observe(n_bits, qt, 5.0)
        g = Gmm_quant(n_components=K, covariance_type=ct, max_iter=3, random_state=0)
        np.random.seed(123)
        try:
            with threadpool_limits(limits=1), contextlib.redirect_stdout(io.StringIO()):
                g.fit(h=y[:300], n_bits=n_bits, sigma2=10 ** -0.5, quantizer=quantizer, quant_type=qt, blocks=blocks,
                      zero_mean=True)
            kind, msg = "ok", ""
        except Exception as exc:  # recorded as data: type name and message
            kind, msg = type(exc).__name__, str(exc)
        out[tag + "__cfg"] = np.array([float(n_bits), K])
        out[tag + "__ctype"] = np.array(ct)
        out[tag + "__kind"] = np.array(kind)
        out[tag + "__msg"] = np.array(msg)
        etags.append(tag)
        print(tag, kind, msg)
    out["tags"] = np.array(tags)
    out["etags"] = np.array(etags)
    np.savez_compressed(os.path.join(HERE, "quant_fit_struct.npz"), **out)
    print("wrote quant_fit_struct.npz:", tags)


if __name__ == "__main__":
    main()
