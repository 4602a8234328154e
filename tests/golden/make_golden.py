"""Generate the golden fixtures for the Bussgang-GMM estimate path.

Runs ONLY in the build container, where the reference checkout exists at
/root/reference.  It imports the reference (read-only, no bytecode written),
fits a few small models with the reference's own EM, runs the reference's
``Gmm_nbit.estimate_from_y`` / ``predict_proba_cplx`` / ``_predict_cplx`` on
fixed observations and stores inputs, intermediates and outputs as ``.npz``
data files next to this script.  Nothing from the reference ships: the
fixtures are numbers only.

Harness-side shims (never applied to reference files, only to the imported
modules in this process) for numpy-2 / sklearn-1.7 API drift, see SURVEY.md
§8(c) C1:
  1. ``np.infty`` alias (gmm_cplx_bussgang.py:494,506)
  2. ``GaussianMixture._check_n_features`` (removed in sklearn 1.7; :487)
  3. ``BaseMixture._print_verbose_msg_init_end`` default ``init_has_converged`` (:523)

The reference's noise RNG is unseeded (utils.py:13, 241-251), so observations
are generated here with an explicit seeded generator using the same model
(y = quant(A h + 10^(-snr/20) CN(0,1))) and stored explicitly.

Usage:  python -B tests/golden/make_golden.py
"""
import os
import sys

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def _import_reference():
    if not os.path.isdir(REF):
        raise SystemExit("make_golden.py: /root/reference is absent; fixtures are committed, nothing to do")
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import numpy as np
    np.infty = np.inf  # shim 1
    from sklearn.mixture import GaussianMixture
    from sklearn.mixture import _base as mixture_base

    def _check_n_features(self, X, reset):  # shim 2
        self.n_features_in_ = X.shape[1]

    GaussianMixture._check_n_features = _check_n_features
    orig = mixture_base.BaseMixture._print_verbose_msg_init_end

    def _init_end(self, lb, init_has_converged=True):  # shim 3
        return orig(self, lb, init_has_converged)

    mixture_base.BaseMixture._print_verbose_msg_init_end = _init_end
    from modules import gmm_cplx_bussgang, gmm_cplx_quant, utils, lloyd_max_quantizer, uniform_quantizer
    from modules.SCM3GPP.SCMMulti import SCMMulti
    return dict(gmm=gmm_cplx_bussgang, gmmq=gmm_cplx_quant, ut=utils, lloyd=lloyd_max_quantizer,
                uni=uniform_quantizer, SCMMulti=SCMMulti)


def main():
    import warnings
    import numpy as np
    from copy import deepcopy
    R = _import_reference()
    ut, gmm_mod = R["ut"], R["gmm"]
    warnings.simplefilter("ignore")

    # ---------------- quantiser tables (host-side producers) -----------------
    q = {}
    for snr, nb in [(5, 2), (5, 3), (-10, 2), (20, 3)]:
        thr, lab, rho = R["lloyd"].load_quantizer(snr, nb)[snr]
        q[f"lloyd_{nb}_{snr}_thr"], q[f"lloyd_{nb}_{snr}_lab"], q[f"lloyd_{nb}_{snr}_rho"] = thr, lab, np.float64(rho)
    for snr, nb in [(5, 2), (-10, 2), (5, 3), (20, 4)]:
        thr, lab, _ = ut.get_quantizer([snr], nb, "uniform")[snr]
        q[f"uniform_{nb}_{snr}_thr"], q[f"uniform_{nb}_{snr}_lab"] = thr, lab
    for nb in range(1, 9):
        q[f"delta_{nb}"] = np.float64(R["uni"].standard_quantization_step(nb))
    # Bussgang gains on a fixed diagonal (KATs for the gain formulas)
    dg = np.array([1.0 + 10 ** -0.5, 0.3, 2.7, 1.0], dtype=float)
    Cy = np.diag(dg).astype(complex)
    q["gain_diag"] = dg
    q["gain_uniform_2_5"] = np.diag(R["uni"].get_Bussgang_matrix(5, 2, Cy)).real
    q["gain_uniform_3_m10"] = np.diag(R["uni"].get_Bussgang_matrix(-10, 3, Cy)).real
    q["gain_lloyd_3_5"] = np.diag(R["lloyd"].get_Bussgang_matrix(3, Cy, R["lloyd"].load_quantizer(5, 3)[5])).real
    q["gain_lloyd_2_5"] = np.diag(R["lloyd"].get_Bussgang_matrix(2, Cy, R["lloyd"].load_quantizer(5, 2)[5])).real
    # quantiser KAT on fixed inputs (utils.py:189-203)
    rng = np.random.default_rng(7)
    zin = np.sqrt(0.5) * (rng.standard_normal((5, 6)) + 1j * rng.standard_normal((5, 6)))
    q["quant_in"] = zin
    q["quant_1"] = ut.quant(zin, 1)
    q["quant_uniform_2_5"] = ut.quant(zin, 2, q["uniform_2_5_thr"], q["uniform_2_5_lab"])
    q["quant_lloyd_3_5"] = ut.quant(zin, 3, q["lloyd_3_5_thr"], q["lloyd_3_5_lab"])
    # pilot matrices (utils.py:337-367)
    q["pilot_8_2_angle_amp"] = ut.get_pilot_matrix(8, 2, 1, "angle_amp")
    q["pilot_8_3_angle_amp"] = ut.get_pilot_matrix(8, 3, 2, "angle_amp")
    # SCM channel generator KAT (SCMMulti.py:30-56, scm_helper.py:39-84)
    h_scm, t_scm = R["SCMMulti"](path_sigma=2.0, n_path=3).generate_channel(4, 1, 16, np.random.default_rng(99))
    q["scm_h"], q["scm_t"] = h_scm, t_scm
    np.savez_compressed(os.path.join(HERE, "quantizers.npz"), **q)
    print("wrote quantizers.npz")

    # ---------------- models --------------------------------------------------
    scm = R["SCMMulti"](path_sigma=2.0, n_path=1)
    h_all, _ = scm.generate_channel(2000 + 512, 1, 32, np.random.default_rng(1234))
    h_all = np.squeeze(h_all).astype(complex)
    h_train, h_val = h_all[:2000], h_all[2000:]

    models = {}
    for name, cov_type, blocks, zero_mean in [("full", "full", None, True),
                                              ("fullmean", "full", None, False),
                                              ("circ", "circulant", None, True),
                                              ("bcirc", "block-circulant", (4, 8), True)]:
        g = gmm_mod.Gmm_nbit(n_components=16, covariance_type=cov_type, random_state=0, max_iter=20)
        g.fit(h_train, blocks=blocks, zero_mean=zero_mean)
        models[name] = (g, h_val)

    # synthetic K=8, N=64 full model (Toeplitz covariances from SCM first rows)
    K8, N64 = 8, 64
    _, t8 = R["SCMMulti"](path_sigma=2.0, n_path=3).generate_channel(K8, 1, N64, np.random.default_rng(42))
    covs = np.stack([ut.toeplitz(t8[k].astype(complex)).T + 1e-6 * np.eye(N64) for k in range(K8)])
    w = np.random.default_rng(11).dirichlet(np.ones(K8))
    gs = gmm_mod.Gmm_nbit(n_components=K8, covariance_type="full")
    gs.means_cplx = np.zeros((K8, N64), dtype=complex)
    gs.covs_cplx = covs
    gs.gm.weights_ = w
    h64, _ = R["SCMMulti"](path_sigma=2.0, n_path=3).generate_channel(64, 1, N64, np.random.default_rng(1002))
    models["synth64"] = (gs, np.squeeze(h64).astype(complex))

    # ---------------- cases ---------------------------------------------------
    # (tag, n_bits, qtype, snr, n_pilots, B)
    base_cases = [("b1_m10", 1, "uniform", -10, 1), ("b1_5", 1, "uniform", 5, 1), ("b1_20", 1, "uniform", 20, 1),
                  ("u2_5", 2, "uniform", 5, 1), ("u2_m10", 2, "uniform", -10, 1), ("l3_5", 3, "lloyd", 5, 1),
                  ("l3_20", 3, "lloyd", 20, 1), ("inf_5", np.inf, "uniform", 5, 1)]
    extra_full = [("p2_b1_5", 1, "uniform", 5, 2), ("p2_u2_5", 2, "uniform", 5, 2), ("l2_m10", 2, "lloyd", -10, 1)]
    modes = {"all": "all", "top1": 1, "top3": 3, "p09": 0.9}
    keep_intermediates = {("full", "b1_5"), ("full", "u2_5"), ("full", "l3_5"), ("full", "inf_5"),
                          ("fullmean", "b1_5"), ("full", "p2_b1_5"), ("synth64", "b1_5")}

    for mname, (g, h_src) in models.items():
        K = g.covs_cplx.shape[0]
        N = g.covs_cplx.shape[-1]
        B = 64 if N <= 32 else 32
        out = {"means_cplx": np.asarray(g.means_cplx, dtype=complex), "covs_cplx": np.asarray(g.covs_cplx),
               "weights": np.asarray(g.gm.weights_, dtype=float), "K": K, "N": N}
        cases = base_cases + (extra_full if mname == "full" else [])
        case_tags = []
        for ci, (tag, n_bits, qtype, snr, n_pilots) in enumerate(cases):
            rng = np.random.default_rng(5000 + 17 * ci + len(mname))
            h = h_src[:B]
            A = ut.get_pilot_matrix(N, n_pilots, n_bits, "angle_amp")
            if n_bits == np.inf:
                quantizer = (None, None, None)
            elif n_bits == 1:
                quantizer = (None, None, None)
            elif qtype == "uniform":
                quantizer = ut.get_quantizer([snr], n_bits, "uniform")[snr]
            else:
                quantizer = R["lloyd"].load_quantizer(snr, n_bits)[snr]
            y = A @ h.T
            y = y.T
            noise = np.sqrt(0.5) * (rng.standard_normal(y.shape) + 1j * rng.standard_normal(y.shape))
            y = y + 10 ** (-snr / 20) * noise
            if n_bits != np.inf:
                y = ut.quant(y, n_bits, quantizer[0], quantizer[1])
            pfx = f"{tag}__"
            out[pfx + "y"] = y
            out[pfx + "h"] = h
            out[pfx + "A"] = A
            out[pfx + "snr"] = np.float64(snr)
            out[pfx + "n_bits"] = np.float64(n_bits)
            out[pfx + "qtype"] = np.array(qtype)
            if quantizer[0] is not None:
                out[pfx + "thr"] = np.asarray(quantizer[0], dtype=float)
                out[pfx + "lab"] = np.asarray(quantizer[1], dtype=float)
            for mtag, mode in modes.items():
                gc = deepcopy(g)
                hest = gc.estimate_from_y(y, snr, N, A, mode, n_bits, qtype, quantizer)
                out[pfx + "hest_" + mtag] = hest
                if mtag == "all":
                    # state after estimate: observation-domain model of this SNR
                    out[pfx + "lp"] = gc._estimate_weighted_log_prob(y)
                    out[pfx + "proba"] = gc.predict_proba_cplx(y)
                    out[pfx + "labels"] = gc._predict_cplx(y)
                    if (mname, tag) in keep_intermediates:
                        _, Cr_inv, Cy, A_eff = deepcopy(g)._prepare_for_prediction(y, A, snr, n_bits, qtype, quantizer)
                        # per-component tables kept for the first two components only (fixture size)
                        out[pfx + "Cy"] = Cy[:2]
                        out[pfx + "Cr"] = gc.gm.covariances_[:2]
                        out[pfx + "P"] = gc.gm.precisions_cholesky_[:2]
                        out[pfx + "Cr_inv"] = Cr_inv[:2]
                        out[pfx + "A_eff"] = A_eff[:2]
                        out[pfx + "means_y"] = gc.gm.means_
            case_tags.append(tag)
        # Gmm_quant twin on one case (gmm_cplx_quant.py:190-267): same tables, same output
        if mname == "full":
            gq = R["gmmq"].Gmm_quant(n_components=K, covariance_type="full")
            gq.means_cplx, gq.covs_cplx, gq.gm.weights_ = g.means_cplx, g.covs_cplx, g.gm.weights_
            gq.gm.covariance_type = "full"
            y = out["u2_5__y"]
            qz = ut.get_quantizer([5], 2, "uniform")[5]
            try:
                out["quant_twin__hest_all"] = gq.estimate_from_y(y, 5, N, out["u2_5__A"], "all", 2, "uniform", qz)
            except Exception as exc:  # pragma: no cover - recorded, not fatal
                print("Gmm_quant twin failed:", exc)
            # K=1 squeeze path (:256-264) and B=1
            g1 = gmm_mod.Gmm_nbit(n_components=1, covariance_type="full")
            g1.means_cplx = g.means_cplx[:1].copy()
            g1.covs_cplx = g.covs_cplx[:1].copy()
            g1.gm.weights_ = np.array([1.0])
            y1 = out["b1_5__y"]
            out["k1__hest_all"] = deepcopy(g1).estimate_from_y(y1, 5, N, None, "all", 1, "uniform", (None, None, None))
            out["b1row__hest_all"] = deepcopy(g).estimate_from_y(y1[:1], 5, N, None, "all", 1, "uniform", (None, None, None))
        out["cases"] = np.array(case_tags)
        path = os.path.join(HERE, f"model_{mname}.npz")
        np.savez_compressed(path, **out)
        print("wrote", path, os.path.getsize(path) // 1024, "KiB")


if __name__ == "__main__":
    main()
