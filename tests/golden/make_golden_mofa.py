"""Generate tests/golden/mofa.npz: golden vectors for the MFA Bussgang estimator (SURVEY.md §8(f) 3;
reference modules/mofa_cplx_bussgang.py:117-216 estimate_from_y / _prepare_for_prediction / _lmmse,
:342-368 predict_proba / predict_proba_max).

Runs ONLY in the build container (reference imported read-only, no bytecode written, the shims of
make_golden.py).  Fits a small MFA with the reference's own EM on SCM channels, then stores the fitted
parameters (means, covs = Lambda Lambda^H + Psi, amps, lambdas, psis), observations y and the
reference's estimates for the four modes at 1-bit / 2-bit uniform / 3-bit Lloyd / inf, plus
predict_proba on the channel-domain model.

Usage:  python -B tests/golden/make_golden_mofa.py
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
    ut = R["ut"]
    np.Inf = np.inf  # mofa_cplx_bussgang.py:302 (numpy 2 removed the alias)
    from modules.mofa_cplx_bussgang import Mofa
    warnings.simplefilter("ignore")
    scm = R["SCMMulti"](path_sigma=2.0, n_path=1)
    h, _ = scm.generate_channel(1600, 1, 16, np.random.default_rng(2024))
    h = np.squeeze(h).astype(complex)
    h_train, h_val = h[:1400], h[1400:]
    np.random.seed(0)  # the reference's MFA initialisation draws from numpy's global RNG
    m = Mofa(n_components=4, latent_dim=4, maxiter=15, verbose=False)
    m.fit(h_train, zero_mean=True)
    out = dict(means=m.means, covs=m.covs, amps=np.asarray(m.amps), lambdas=m.lambdas, psis=m.psis, h_val=h_val)
    out["proba_chan"] = m.predict_proba(h_val[:50])
    tags = []
    rng = np.random.default_rng(31)
    for tag, snr, nb, qtype in [("b1", 5.0, 1, "uniform"), ("b2u", 5.0, 2, "uniform"), ("b3l", 0.0, 3, "lloyd"),
                                ("inf", 10.0, np.inf, "uniform")]:
        quantizer = ut.get_quantizer([snr], nb, qtype)[snr] if nb not in (1, np.inf) else (None, None, None)
        w = (rng.standard_normal(h_val.shape) + 1j * rng.standard_normal(h_val.shape)) * np.sqrt(0.5)
        y = h_val + 10 ** (-snr / 20) * w
        if nb != np.inf:
            y = ut.quant(y, nb, quantizer[0], quantizer[1])
        p = tag + "__"
        out[p + "y"] = y
        out[p + "snr"] = np.float64(snr)
        out[p + "n_bits"] = np.float64(nb)
        out[p + "qtype"] = np.array(qtype)
        if quantizer[0] is not None:
            out[p + "thr"], out[p + "lab"] = np.asarray(quantizer[0]), np.asarray(quantizer[1])
        for mname, mode in [("all", "all"), ("top1", 1), ("top3", 3), ("p09", 0.9)]:
            out[p + "h_" + mname] = m.estimate_from_y(y, snr, None, mode, nb, qtype, quantizer)
        out[p + "proba_obs"] = m.predict_proba(y)
        tags.append(tag)
    out["tags"] = np.array(tags)
    np.savez_compressed(os.path.join(HERE, "mofa.npz"), **out)
    print("wrote mofa.npz:", tags)


if __name__ == "__main__":
    main()
