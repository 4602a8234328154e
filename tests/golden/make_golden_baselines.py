"""Generate tests/golden/baselines.npz: golden vectors for the global / genie Bussgang-LMMSE baselines
(reference estimators/blmmse.py:20-97).

Runs ONLY in the build container (reference imported read-only, no bytecode written).  SCM channels
with their Toeplitz first rows t (SCMMulti.generate_channel), a sample covariance as the global C
(as Bussgang_GMM.py:131-139 builds it from training channels), fixed noise draws, and the reference's
BLMMSE(snr).estimate_global / estimate_genie and LS(snr) (estimators/LS.py) outputs for 1-bit, 2-bit uniform, 3-bit Lloyd-Max and
n_bits = inf, with A = I and a 2-pilot A.

Usage:  python -B tests/golden/make_golden_baselines.py
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
    sys.path.insert(0, "/root/reference")
    from estimators.blmmse import BLMMSE
    from estimators.LS import LS
    warnings.simplefilter("ignore")
    N = 16
    scm = R["SCMMulti"](path_sigma=2.0, n_path=3)
    h_tr, _ = scm.generate_channel(2000, 1, N, np.random.default_rng(71))
    h_tr = np.squeeze(h_tr).astype(complex)
    C = (h_tr.T @ h_tr.conj()) / h_tr.shape[0]
    h, t = scm.generate_channel(120, 1, N, np.random.default_rng(72))
    h = np.squeeze(h).astype(complex)
    out = dict(C=C, h=h, t=t)
    rng = np.random.default_rng(73)
    A2 = ut.get_pilot_matrix(N, 2, 1, "angle_amp")
    tags = []
    for tag, snr, nb, qt, A in [("b1", 5.0, 1, "uniform", None), ("b2u", 5.0, 2, "uniform", None),
                                ("b3l", 0.0, 3, "lloyd", None), ("inf", 10.0, np.inf, "uniform", None),
                                ("b1_A2", 5.0, 1, "uniform", A2), ("b2u_A2", 10.0, 2, "uniform", A2)]:
        quantizer = ut.get_quantizer([snr], nb, qt)[snr] if nb not in (1, np.inf) else (None, None, None)
        y0 = h if A is None else (A @ h.T).T
        w = (rng.standard_normal(y0.shape) + 1j * rng.standard_normal(y0.shape)) * np.sqrt(0.5)
        y = y0 + 10 ** (-snr / 20) * w
        if nb != np.inf:
            y = ut.quant(y, nb, quantizer[0], quantizer[1])
        est = BLMMSE(snr)
        p = tag + "__"
        out[p + "y"] = y
        out[p + "snr"] = np.float64(snr)
        out[p + "n_bits"] = np.float64(nb)
        out[p + "qtype"] = np.array(qt)
        out[p + "A"] = np.zeros((0, 0), complex) if A is None else np.asarray(A, complex)
        if quantizer[0] is not None:
            out[p + "thr"], out[p + "lab"] = np.asarray(quantizer[0]), np.asarray(quantizer[1])
        out[p + "h_global"] = est.estimate_global(y, C, A, nb, qt, quantizer)
        out[p + "h_genie"] = est.estimate_genie(y, t, A, nb, qt, quantizer)
        ls = LS(snr)
        out[p + "ls_global"] = ls.estimate_global(y, C, A, nb, qt, quantizer)
        if nb != np.inf:  # the reference's genie LS assigns lstsq's tuple for n_bits = inf (LS.py:35-37) and fails
            out[p + "ls_genie"] = ls.estimate_genie(y, t, A, nb, qt, quantizer)
        tags.append(tag)
    out["tags"] = np.array(tags)
    # the scripts' Bussgang pair for the rate bound (Bussgang_GMM.py:148-151): uniform get_Bussgang_matrix
    # and get_Cr (quantised-variance diagonal, uniform_quantizer.py:114-173) for multi-bit quantisers
    from modules.uniform_quantizer import get_Bussgang_matrix, get_Cr
    for tag, snr, nb, qt in [("r2u", 5.0, 2, "uniform"), ("r3l", 0.0, 3, "lloyd"), ("r1", 5.0, 1, "uniform")]:
        quantizer = ut.get_quantizer([snr], nb, qt)[snr]
        Cy = C + 10 ** (-snr / 10) * np.eye(N, dtype=complex)
        out[tag + "__buss"] = np.real(np.diag(get_Bussgang_matrix(snr, nb, Cy)))
        out[tag + "__Cr"] = get_Cr(Cy, nb, snr, quantizer)
    np.savez_compressed(os.path.join(HERE, "baselines.npz"), **out)
    print("wrote baselines.npz:", tags)


if __name__ == "__main__":
    main()
