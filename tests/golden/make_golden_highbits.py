"""Golden vectors for uniform quantisers beyond J. Max's table (n_bits > 8): the reference falls back to the
Hui-Neuhoff asymptotic step 4 sqrt(b) 2^-b (uniform_quantizer.py:6-23, the `else` at :15) in both the quantiser
tables (get_quantizer, utils.py) and the Bussgang gain (uniform_quantizer.py:44-45, 60-72).

Runs ONLY in the build container (imports /root/reference read-only through make_golden.py's harness).  The
observations use the reference's own `quant` on h + seeded noise (its crandn is unseeded, utils.py:13), stored
explicitly.  Writes highbits.npz: per case y, the quantiser tables, and the reference's estimate_from_y for the
modes 'all' and 1, plus predict_proba_cplx after the estimate (the observation-domain state).

Usage:  python -B tests/golden/make_golden_highbits.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def main():
    import warnings
    from copy import deepcopy
    import numpy as np
    from make_golden import _import_reference
    R = _import_reference()
    gmm_mod, ut = R["gmm"], R["ut"]
    warnings.simplefilter("ignore")
    base = np.load(os.path.join(HERE, "model_fullmean.npz"))
    K, N = int(base["K"]), int(base["N"])
    means, covs, w = base["means_cplx"], base["covs_cplx"], base["weights"]
    h = base["b1_5__h"]
    out = dict(means_cplx=means, covs_cplx=covs, weights=w, h=h)
    A = np.eye(N, dtype=complex)
    cases = []
    for nb, snr in ((9, 5), (10, 20), (12, -10), (16, 5)):
        tag = f"u{nb}_{snr}".replace("-", "m")
        thr, lab, rho = ut.get_quantizer([snr], nb, "uniform")[snr]
        rng = np.random.default_rng(4000 + nb)
        noise = (rng.standard_normal(h.shape) + 1j * rng.standard_normal(h.shape)) / np.sqrt(2)
        y = ut.quant(h + 10 ** (-snr / 20) * noise, nb, thr, lab)
        out[tag + "__y"], out[tag + "__thr"], out[tag + "__lab"] = y, thr, lab
        out[tag + "__n_bits"], out[tag + "__snr"] = np.int64(nb), np.float64(snr)
        for mtag, mode in (("all", "all"), ("top1", 1)):
            g = gmm_mod.Gmm_nbit(n_components=K, covariance_type="full")
            g.means_cplx, g.covs_cplx, g.gm.weights_ = means, covs, w
            out[f"{tag}__hest_{mtag}"] = deepcopy(g).estimate_from_y(y, snr, N, A, mode, nb, "uniform",
                                                                      (thr, lab, rho))
        g = gmm_mod.Gmm_nbit(n_components=K, covariance_type="full")
        g.means_cplx, g.covs_cplx, g.gm.weights_ = means, covs, w
        g.estimate_from_y(y, snr, N, A, "all", nb, "uniform", (thr, lab, rho))
        out[tag + "__proba"] = g.predict_proba_cplx(y)
        out[tag + "__means_y"] = np.asarray(g.gm.means_)
        cases.append(tag)
    out["cases"] = np.array(cases)
    np.savez_compressed(os.path.join(HERE, "highbits.npz"), **out)
    print("wrote highbits.npz", cases)


if __name__ == "__main__":
    main()
