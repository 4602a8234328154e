"""The reference's error paths and argument quirks on the estimate path, pinned to its own behaviour
(tests/golden/quirks.npz, made by tests/golden/make_golden_quirks.py from the reference itself):

  * a non positive-definite Cr -> ValueError with the reference's message (gmm_cplx_bussgang.py:43-46),
    at n_bits = inf (Cr = Cy) and at 1 bit (arcsine law of a negative diagonal);
  * an np.int64 mode falls into the cumulative-probability branch (isinstance(.., int) at :197);
  * an unknown multi-bit quantizer_type leaves the Bussgang gain at 0 (:281-284);
  * n_bits = 'inf' (a string) raises the reference's TypeError; a 1-D y its ValueError (:405).
"""
import os

import numpy as np
import pytest

from conftest import ROOT, rel_fro

QUIRKS = os.path.join(ROOT, "tests", "golden", "quirks.npz")


@pytest.fixture(scope="module")
def qx():
    return np.load(QUIRKS)


def _args(qx):
    N = qx["covs_cplx"].shape[-1]
    from quantized_channel_estimation_amd import inputs
    qz = inputs.get_quantizer([5], 2, "uniform")[5]
    return N, qz


# ---- oracle (CPU): the restatement reproduces the quirks --------------------------------------
def test_oracle_quirks(qx):
    from oracle import qce_oracle as O
    N, qz = _args(qx)
    m, c, w, y = qx["means_cplx"], qx["covs_cplx"], qx["weights"], qx["y"]
    for n in (1, 3):
        assert str(qx[f"int64_{n}__kind"]) == "ok"
        h = O.estimate(m, c, w, y, 5, N, None, np.int64(n), 2, "uniform", qz)
        assert rel_fro(h, qx[f"int64_{n}__result"]) < 1e-11
    for mtag, mode in (("all", "all"), ("top1", 1)):
        h = O.estimate(m, c, w, y, 5, N, None, mode, 2, "foo", qz)
        assert rel_fro(h, qx[f"unknown_q_{mtag}__result"]) < 1e-11
    for tag, nb in (("nonpd_inf", np.inf), ("nonpd_b1", 1)):
        assert str(qx[tag + "__kind"]) == "ValueError"
        with pytest.raises(ValueError) as ei:
            O.estimate(m, qx["bad_covs"], w, qx[tag + "__y"], 20, N, None, "all", nb)
        assert str(ei.value) == str(qx[tag + "__result"])


# ---- device path -----------------------------------------------------------------------------
@pytest.mark.gpu
def test_device_nonpd_raises_reference_error(qx):
    from quantized_channel_estimation_amd import Gmm_nbit
    N, _ = _args(qx)
    for tag, nb in (("nonpd_inf", np.inf), ("nonpd_b1", 1)):
        g = Gmm_nbit.from_params(qx["means_cplx"], qx["bad_covs"], qx["weights"])
        with pytest.raises(ValueError) as ei:
            g.estimate_from_y(qx[tag + "__y"], 20, N, None, "all", nb)
        assert str(ei.value) == str(qx[tag + "__result"]), tag
        # the model stays usable: a valid mixture on the same object class estimates normally
        g2 = Gmm_nbit.from_params(qx["means_cplx"], qx["covs_cplx"], qx["weights"])
        assert np.all(np.isfinite(g2.estimate_from_y(qx[tag + "__y"], 20, N, None, "all", nb)))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 3])
def test_device_int64_mode_takes_probability_branch(qx, n):
    from quantized_channel_estimation_amd import Gmm_nbit
    N, qz = _args(qx)
    g = Gmm_nbit.from_params(qx["means_cplx"], qx["covs_cplx"], qx["weights"])
    h = g.estimate_from_y(qx["y"], 5, N, None, np.int64(n), 2, "uniform", qz)
    assert rel_fro(h, qx[f"int64_{n}__result"]) < 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("mtag,mode", [("all", "all"), ("top1", 1)])
def test_device_unknown_quantizer_type(qx, mtag, mode):
    from quantized_channel_estimation_amd import Gmm_nbit
    N, qz = _args(qx)
    g = Gmm_nbit.from_params(qx["means_cplx"], qx["covs_cplx"], qx["weights"])
    h = g.estimate_from_y(qx["y"], 5, N, None, mode, 2, "foo", qz)
    assert rel_fro(h, qx[f"unknown_q_{mtag}__result"]) < 1e-9


@pytest.mark.gpu
def test_device_argument_errors_match_reference(qx):
    from quantized_channel_estimation_amd import Gmm_nbit
    N, qz = _args(qx)
    g = Gmm_nbit.from_params(qx["means_cplx"], qx["covs_cplx"], qx["weights"])
    with pytest.raises(TypeError) as ei:
        g.estimate_from_y(qx["y"], 5, N, None, "all", "inf", "uniform", qz)
    assert str(qx["str_inf__kind"]) == "TypeError" and str(ei.value) == str(qx["str_inf__result"])
    with pytest.raises(ValueError) as ei:
        g.estimate_from_y(qx["y"][0], 5, N, None, "all", 2, "uniform", qz)
    assert str(qx["y1d__kind"]) == "ValueError" and str(ei.value) == str(qx["y1d__result"])
