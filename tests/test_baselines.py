"""Global / genie Bussgang-LMMSE baselines (estimators/blmmse.py:20-97).

CPU: the oracle restatement and the Toeplitz construction against the reference's own outputs in
tests/golden/baselines.npz (make_golden_baselines.py).  GPU: quantized_channel_estimation_amd.baselines
through libqce.so (K=1 model for the global filter; one component per sample + qce_estimate_assigned for
the genie) against the same vectors, 1e-5 relative Frobenius (FP64 path: measured ~1e-12)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, rel_fro


@pytest.fixture(scope="module")
def bl():
    return dict(np.load(os.path.join(GOLDEN, "baselines.npz"), allow_pickle=False))


def _case(bl, tag):
    p = tag + "__"
    nb = float(bl[p + "n_bits"])
    A = bl[p + "A"]
    quantizer = (bl[p + "thr"], bl[p + "lab"], None) if (p + "thr") in bl else (None, None, None)
    return (bl[p + "y"], float(bl[p + "snr"]), (np.inf if np.isinf(nb) else int(nb)), str(bl[p + "qtype"]),
            quantizer, None if A.size == 0 else A)


TAGS = ["b1", "b2u", "b3l", "inf", "b1_A2", "b2u_A2"]


def test_toeplitz_covs_match_scipy(bl):
    from scipy.linalg import toeplitz
    from quantized_channel_estimation_amd.baselines import _toeplitz_covs
    t = bl["t"][:5]
    C = _toeplitz_covs(t)
    for b in range(5):
        assert np.array_equal(C[b], toeplitz(t[b]).T)


@pytest.mark.parametrize("tag", TAGS)
def test_oracle_blmmse_matches_reference(bl, tag):
    from scipy.linalg import toeplitz
    from oracle import qce_oracle as O
    y, snr, nb, qt, quantizer, A = _case(bl, tag)
    N = bl["C"].shape[0]
    Ae = np.eye(N) if A is None else A
    W = O.blmmse_filter(bl["C"], Ae, snr, nb, qt, quantizer)
    assert rel_fro(y @ W.T, bl[tag + "__h_global"]) < 1e-9
    hg = np.stack([O.blmmse_filter(toeplitz(bl["t"][b]).T, Ae, snr, nb, qt, quantizer) @ y[b]
                   for b in range(y.shape[0])])
    assert rel_fro(hg, bl[tag + "__h_genie"]) < 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("tag", TAGS)
def test_gpu_blmmse_matches_reference(bl, tag):
    from quantized_channel_estimation_amd.baselines import BLMMSE, mp_eval
    y, snr, nb, qt, quantizer, A = _case(bl, tag)
    est = BLMMSE(snr, chunk=50)  # several chunks
    hg = est.estimate_global(y, bl["C"], A, nb, qt, quantizer)
    assert rel_fro(hg, bl[tag + "__h_global"]) < 1e-5, tag
    hq = mp_eval(est, y, bl["t"], None, True, A, nb, qt, quantizer)
    assert rel_fro(hq, bl[tag + "__h_genie"]) < 1e-5, tag


@pytest.mark.gpu
@pytest.mark.parametrize("tag", TAGS)
def test_gpu_ls_matches_reference(bl, tag):
    from quantized_channel_estimation_amd.baselines import LS
    y, snr, nb, qt, quantizer, A = _case(bl, tag)
    ls = LS(snr, chunk=50)
    assert rel_fro(ls.estimate_global(y, bl["C"], A, nb, qt, quantizer), bl[tag + "__ls_global"]) < 1e-9, tag
    if (tag + "__ls_genie") in bl:
        assert rel_fro(ls.estimate_genie(y, bl["t"], A, nb, qt, quantizer), bl[tag + "__ls_genie"]) < 1e-9, tag
    else:
        with pytest.raises(ValueError):
            ls.estimate_genie(y, bl["t"], A, nb, qt, quantizer)


def _ls_general_expected(y, covs, A, snr, n_bits):
    """LS.py:21-32 / :55-73 restated for the test: A_eff = sqrt(2/pi) diag(Cy)^-1/2 A (1-bit) or A (inf),
    h = lstsq(A_eff, y) per covariance."""
    out = []
    for C, yb in zip(covs, y):
        Cy = A @ C @ A.conj().T + 10 ** (-0.1 * snr) * np.eye(A.shape[0])
        Ae = A if n_bits == np.inf else np.sqrt(2 / np.pi) * np.diag(1 / np.sqrt(np.real(np.diag(Cy)))) @ A
        out.append(np.linalg.lstsq(Ae, yb.T, rcond=None)[0].T)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("n_bits", [1, np.inf])
def test_gpu_ls_general_pilot_matrix(bl, n_bits):
    """LS with a dense, non-column-orthogonal pilot matrix (M = 2N rows): device pseudo-inverse vs lstsq."""
    from quantized_channel_estimation_amd.baselines import LS, _toeplitz_covs
    rng = np.random.default_rng(7)
    C = bl["C"]
    N = C.shape[0]
    M = 2 * N
    A = (rng.standard_normal((M, N)) + 1j * rng.standard_normal((M, N))) / np.sqrt(2 * M)
    B = 40
    y = (np.sign(rng.standard_normal((B, M))) + 1j * np.sign(rng.standard_normal((B, M)))) / np.sqrt(2)
    snr = 5.0
    ls = LS(snr, chunk=16)
    hg = ls.estimate_global(y, C, A, n_bits)
    exp_g = _ls_general_expected([y], [C], A, snr, n_bits)[0]
    assert rel_fro(hg, exp_g) < 1e-9
    if n_bits == 1:
        t = bl["t"][:B]
        covs = _toeplitz_covs(t)
        hq = ls.estimate_genie(y, t, A, n_bits)
        exp_q = np.stack([_ls_general_expected([y[b:b + 1]], [covs[b]], A, snr, n_bits)[0][0] for b in range(B)])
        assert rel_fro(hq, exp_q) < 1e-9


def test_ls_kind_routes_pilot_matrices():
    from quantized_channel_estimation_amd.baselines import _ls_kind
    assert _ls_kind(None) is True
    assert _ls_kind(np.kron(np.array([[1.0], [1j]]), np.eye(4))) is True
    rng = np.random.default_rng(0)
    assert _ls_kind(rng.standard_normal((8, 4)) + 0j) == "general"
    with pytest.raises(NotImplementedError):
        _ls_kind(rng.standard_normal((3, 4)) + 0j)


@pytest.mark.gpu
def test_gpu_ls_general_ill_conditioned_and_rank_deficient(bl):
    """Gram-matrix pivots (qce_genie.hip k_ls_pinv): an ill-conditioned pilot matrix (cond ~1e4, unquantised,
    30 dB) still matches lstsq; a rank-deficient one (two equal columns), where lstsq returns the
    minimum-norm solution, is refused with ValueError instead of returning inf / NaN."""
    from quantized_channel_estimation_amd.baselines import LS
    rng = np.random.default_rng(11)
    C = bl["C"]
    N = C.shape[0]
    M = 2 * N
    U, _ = np.linalg.qr(rng.standard_normal((M, N)) + 1j * rng.standard_normal((M, N)))
    V, _ = np.linalg.qr(rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N)))
    A = U @ np.diag(np.logspace(0, -4, N)) @ V.conj().T
    y = rng.standard_normal((30, M)) + 1j * rng.standard_normal((30, M))
    ls = LS(30.0, chunk=16)
    hg = ls.estimate_global(y, C, A, np.inf)
    exp = _ls_general_expected([y], [C], A, 30.0, np.inf)[0]
    assert rel_fro(hg, exp) < 1e-6  # Gauss-Jordan on A^H A: error ~ cond(A)^2 eps
    A2 = A.copy()
    A2[:, 1] = A2[:, 0]
    with pytest.raises(ValueError, match="full column rank"):
        ls.estimate_global(y, C, A2, np.inf)
