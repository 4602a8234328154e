"""Golden vectors for the reference's error paths and argument quirks on the estimate path.

Runs ONLY in the build container (imports /root/reference read-only through make_golden.py's
harness; nothing from the reference ships).  Writes quirks.npz: for each case the inputs, and
either the reference's output or the exception type and message it raised.

Cases (SURVEY.md §7 hard part 6, §5 failure detection):
  * nonpd_inf:  a covariance with a negative eigenvalue, n_bits = inf -> Cr = Cy not positive
                definite -> compute_precision_cholesky's LinAlgError -> ValueError(msg)
                (gmm_cplx_bussgang.py:43-46)
  * nonpd_b1:   the same model at 1 bit: a negative diagonal makes the arcsine law NaN (:292-301)
  * int64_mode: n_summands_or_proba = np.int64(3) / np.int64(1) take the float-p branch (:197, :229-242)
  * unknown_q:  multi-bit with quantizer_type 'foo' leaves A_buss = 0 (:281-284)
  * str_inf:    n_bits = 'inf' (a string) in _prepare_for_prediction (:276-285)
  * y1d:        a 1-D observation vector (:405)

Usage:  python -B tests/golden/make_golden_quirks.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def _run(fn):
    try:
        return ("ok", fn())
    except Exception as exc:  # recorded as data: type name and message
        return (type(exc).__name__, str(exc))


def main():
    import warnings
    from copy import deepcopy
    import numpy as np
    from make_golden import _import_reference
    R = _import_reference()
    gmm_mod, ut = R["gmm"], R["ut"]
    warnings.simplefilter("ignore")
    out = {}
    base = np.load(os.path.join(HERE, "model_fullmean.npz"))
    K, N = int(base["K"]), int(base["N"])

    def model(means, covs, w):
        g = gmm_mod.Gmm_nbit(n_components=covs.shape[0], covariance_type="full")
        g.means_cplx, g.covs_cplx, g.gm.weights_ = means, covs, w
        return g

    means, covs, w = base["means_cplx"], base["covs_cplx"], base["weights"]
    y = base["u2_5__y"]
    A = np.eye(N, dtype=complex)
    out["means_cplx"], out["covs_cplx"], out["weights"], out["y"] = means, covs, w, y

    # non-PD covariance: component 1 gets a negative eigenvalue (-3 on the first axis)
    bad = covs.copy()
    bad[1] = bad[1] - 3.5 * np.outer(np.eye(N)[0], np.eye(N)[0])
    out["bad_covs"] = bad
    for tag, nb in (("nonpd_inf", np.inf), ("nonpd_b1", 1)):
        yq = base["b1_5__y"] if nb == 1 else base["inf_5__y"]
        out[tag + "__y"] = yq
        kind, val = _run(lambda: model(means, bad, w).estimate_from_y(yq, 20, N, A, "all", nb, "uniform",
                                                                     (None, None, None)))
        out[tag + "__kind"] = np.array(kind)
        out[tag + "__result"] = np.array(val) if kind != "ok" else val

    # np.int64 modes
    qz = ut.get_quantizer([5], 2, "uniform")[5]
    for n in (1, 3):
        kind, val = _run(lambda: deepcopy(model(means, covs, w)).estimate_from_y(y, 5, N, A, np.int64(n), 2, "uniform",
                                                                                 qz))
        out[f"int64_{n}__kind"] = np.array(kind)
        out[f"int64_{n}__result"] = val
    # unknown multi-bit quantiser type
    for mtag, mode in (("all", "all"), ("top1", 1)):
        kind, val = _run(lambda: deepcopy(model(means, covs, w)).estimate_from_y(y, 5, N, A, mode, 2, "foo", qz))
        out[f"unknown_q_{mtag}__kind"] = np.array(kind)
        out[f"unknown_q_{mtag}__result"] = val
    # n_bits given as the string 'inf'
    kind, val = _run(lambda: deepcopy(model(means, covs, w)).estimate_from_y(y, 5, N, A, "all", "inf", "uniform", qz))
    out["str_inf__kind"], out["str_inf__result"] = np.array(kind), np.array(str(val))
    # 1-D observation
    kind, val = _run(lambda: deepcopy(model(means, covs, w)).estimate_from_y(y[0], 5, N, A, "all", 2, "uniform", qz))
    out["y1d__kind"], out["y1d__result"] = np.array(kind), np.array(str(val))
    for k, v in out.items():
        if k.endswith("__kind"):
            print(k, v)
    np.savez_compressed(os.path.join(HERE, "quirks.npz"), **out)
    print("wrote quirks.npz")


if __name__ == "__main__":
    main()
