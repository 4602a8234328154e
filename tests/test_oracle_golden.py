"""The CPU oracle pinned against fixtures produced by the reference itself (tests/golden/make_golden.py)."""
import numpy as np
import pytest

import os

from conftest import MODELS, MODES, ROOT, case_args, rel_fro
from oracle import qce_oracle as O


@pytest.mark.parametrize("mname", MODELS)
def test_oracle_estimate_all_cases(golden_models, mname):
    fx = golden_models[mname]
    for tag in fx["cases"]:
        tag = str(tag)
        y, snr, N, A, n_bits, qtype, quantizer = case_args(fx, tag)
        for mtag, mode in MODES.items():
            h = O.estimate(fx["means_cplx"], fx["covs_cplx"], fx["weights"], y, snr, N, A, mode, n_bits, qtype, quantizer)
            ref = fx[f"{tag}__hest_{mtag}"]
            assert rel_fro(h, ref) < 1e-11, (mname, tag, mtag, rel_fro(h, ref))


@pytest.mark.parametrize("mname", MODELS)
def test_oracle_logprob_proba_labels(golden_models, mname):
    fx = golden_models[mname]
    for tag in fx["cases"]:
        tag = str(tag)
        y, snr, N, A, n_bits, qtype, quantizer = case_args(fx, tag)
        t = O.prepare(fx["means_cplx"], fx["covs_cplx"], A, snr, n_bits, qtype, quantizer)
        lp = O.weighted_log_prob(y, t["means_y"], t["P"], fx["weights"])
        np.testing.assert_allclose(lp, fx[f"{tag}__lp"], rtol=1e-12, atol=1e-9)
        np.testing.assert_allclose(O.predict_proba(y, t["means_y"], t["P"], fx["weights"]), fx[f"{tag}__proba"],
                                   rtol=1e-9, atol=1e-14)
        np.testing.assert_array_equal(O.predict(y, t["means_y"], t["P"], fx["weights"]), fx[f"{tag}__labels"])


def test_oracle_intermediates(golden_models):
    n = 0
    for mname in MODELS:
        fx = golden_models[mname]
        for tag in fx["cases"]:
            tag = str(tag)
            if f"{tag}__Cy" not in fx:
                continue
            y, snr, N, A, n_bits, qtype, quantizer = case_args(fx, tag)
            t = O.prepare(fx["means_cplx"], fx["covs_cplx"], A, snr, n_bits, qtype, quantizer)
            for key, ours in [("Cy", t["Cy"][:2]), ("Cr", t["Cr"][:2]), ("P", t["P"][:2]),
                              ("Cr_inv", t["Cr_inv"][:2]), ("A_eff", t["A_eff"][:2]), ("means_y", t["means_y"])]:
                assert rel_fro(ours, fx[f"{tag}__{key}"]) < 1e-12, (mname, tag, key)
            n += 1
    assert n >= 6


def test_oracle_loop_equals_vectorised(golden_models):
    fx = golden_models["fullmean"]
    y, snr, N, A, n_bits, qtype, quantizer = case_args(fx, "u2_5")
    h1 = O.estimate_loop(fx["means_cplx"], fx["covs_cplx"], fx["weights"], y[:16], snr, N, A, n_bits, qtype, quantizer)
    assert rel_fro(h1, fx["u2_5__hest_all"][:16]) < 1e-12


def test_oracle_special_cases(golden_models):
    fx = golden_models["full"]
    y = fx["b1_5__y"]
    N = int(fx["N"])
    h = O.estimate(fx["means_cplx"][:1], fx["covs_cplx"][:1], np.array([1.0]), y, 5.0, N, None, "all", 1)
    assert rel_fro(h, fx["k1__hest_all"]) < 1e-12
    h = O.estimate(fx["means_cplx"], fx["covs_cplx"], fx["weights"], y[:1], 5.0, N, None, "all", 1)
    assert rel_fro(h, fx["b1row__hest_all"]) < 1e-12
    # Gmm_quant twin (gmm_cplx_quant.py:190-267) equals Gmm_nbit on the same parameters
    assert rel_fro(fx["quant_twin__hest_all"], fx["u2_5__hest_all"]) < 1e-13


def test_oracle_gain_kats():
    q = dict(np.load("tests/golden/quantizers.npz"))
    d = q["gain_diag"]
    np.testing.assert_allclose(O.gain_uniform(5, 2, d).real, q["gain_uniform_2_5"], rtol=1e-14)
    np.testing.assert_allclose(O.gain_uniform(-10, 3, d).real, q["gain_uniform_3_m10"], rtol=1e-14)
    np.testing.assert_allclose(O.gain_lloyd(3, d, q["lloyd_3_5_thr"], q["lloyd_3_5_lab"]).real, q["gain_lloyd_3_5"],
                               rtol=1e-14)
    # 1-bit gain sqrt(2/pi)/sqrt(Cy_ii) at Cy_ii = 1 + 10^-0.5 (SURVEY §4 KAT)
    assert abs(np.sqrt(2 / np.pi) / np.sqrt(d[0]) - 0.69546) < 5e-6
    for nb in range(1, 9):
        assert O.standard_step(nb) == q[f"delta_{nb}"]
    np.testing.assert_array_equal(O.quant(q["quant_in"], 1), q["quant_1"])
    np.testing.assert_array_equal(O.quant(q["quant_in"], 3, q["lloyd_3_5_thr"], q["lloyd_3_5_lab"]), q["quant_lloyd_3_5"])


def test_cpu_baseline_timing_recorded():
    """the loop-faithful oracle bench.py times as the CPU baseline runs within +-15% of the
    reference's own estimate_from_y (and gives identical results) — measured in the build container by
    tests/golden/time_reference.py, recorded in timing_ratio.json."""
    import json
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "timing_ratio.json")))
    for cfg in ("cfg1", "cfg2"):
        assert 0.85 <= d[cfg]["ratio"] <= 1.15, (cfg, d[cfg]["ratio"])
        assert d[cfg]["rel_fro"] < 1e-12
