"""Generate tests/golden/quant_fit.npz: golden fits of the reference's Gmm_quant (EM on quantised
observations with covariance recovery; gmm_cplx_quant.py:103-189 fit, :459-602 fit_predict /
_initialize_parameters / _initialize, :640-731 E/M steps, :732-854 estimate_gaussian_parameters /
estimate_gaussian_covariances_full; cov_est_quant.py:31-88; utils.py:651-700).

Runs ONLY in the build container (reference imported read-only, no bytecode written, the shims of
make_golden.py).  Training data: SCM channels observed as y = Q(h + sigma w) with the reference's own
quant (noise drawn here with a seeded generator, since the reference's is unseeded).  K-means runs with one
thread (sklearn sums threaded centre partials in completion order); numpy's global RNG is seeded before each
fit (the Gauss-Newton solver of cov_est_quant draws from it when an iterate leaves [0.1, 10]).

Usage:  python -B tests/golden/make_golden_quant_fit.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

CASES = [  # tag, n_bits, quantizer type, zero_mean, K, max_iter, snr
    ("b1_zm", 1, "uniform", True, 3, 8, 5.0),
    ("b2u_zm", 2, "uniform", True, 3, 8, 5.0),
    ("b3l_zm", 3, "lloyd", True, 3, 6, 10.0),
    ("inf_mean", "inf", "uniform", False, 3, 8, 10.0),
    ("b1_mean", 1, "uniform", False, 2, 6, 0.0),
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
    h, _ = scm.generate_channel(1500, 1, 8, np.random.default_rng(5))
    h = np.squeeze(h).astype(complex)
    out = dict(h=h)
    rng = np.random.default_rng(6)
    tags = []
    for tag, nb, qt, zm, K, max_iter, snr in CASES:
        n_bits = np.inf if nb == "inf" else nb
        quantizer = ut.get_quantizer([snr], n_bits, qt)[snr] if n_bits not in (1, np.inf) else (None, None, None)
        w = (rng.standard_normal(h.shape) + 1j * rng.standard_normal(h.shape)) * np.sqrt(0.5)
        y = h + 10 ** (-snr / 20) * w
        if n_bits != np.inf:
            y = ut.quant(y, n_bits, quantizer[0], quantizer[1])
        sigma2 = 10 ** (-snr / 10)
        g = Gmm_quant(n_components=K, covariance_type="full", max_iter=max_iter, random_state=0)
        np.random.seed(123)
        with threadpool_limits(limits=1):
            g.fit(h=y, n_bits=n_bits, sigma2=sigma2, quantizer=quantizer, quant_type=qt, zero_mean=zm)
        p = tag + "__"
        out[p + "y"] = y
        out[p + "cfg"] = np.array([float(n_bits), float(zm), K, max_iter, snr, sigma2])
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
        tags.append(tag)
    out["tags"] = np.array(tags)
    np.savez_compressed(os.path.join(HERE, "quant_fit.npz"), **out)
    print("wrote quant_fit.npz:", tags)


if __name__ == "__main__":
    main()
