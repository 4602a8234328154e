"""HIP path vs the reference (golden fixtures) and vs the CPU oracle, through the C-ABI.

Tolerances (BASELINE.json north_star): channel estimates within 1e-5 relative Frobenius of the
reference; argmax component indices bit-exact; FP64 tables (Cy, Cr, P, ...) within 1e-10.
"""
import copy
import pickle

import numpy as np
import pytest

from conftest import MODELS, MODES, case_args, rel_fro

pytestmark = pytest.mark.gpu

H_TOL = 1e-5


def _gpu_or_skip():
    from quantized_channel_estimation_amd import _lib
    if _lib.device_count() == 0:
        pytest.fail("no GPU visible for a gpu-marked test")


def _model(fx, cls=None):
    from quantized_channel_estimation_amd import Gmm_nbit
    cls = cls or Gmm_nbit
    return cls.from_params(fx["means_cplx"], fx["covs_cplx"], fx["weights"])


@pytest.mark.parametrize("mname", MODELS)
def test_estimate_matches_reference_all_modes(golden_models, mname):
    _gpu_or_skip()
    fx = golden_models[mname]
    g = _model(fx)
    worst = {}
    for tag in fx["cases"]:
        tag = str(tag)
        y, snr, N, A, n_bits, qtype, quantizer = case_args(fx, tag)
        for mtag, mode in MODES.items():
            h = g.estimate_from_y(y, snr, N, A, mode, n_bits, qtype, quantizer)
            ref = fx[f"{tag}__hest_{mtag}"]
            err = rel_fro(h, ref)
            worst[(tag, mtag)] = err
            assert err < H_TOL, (mname, tag, mtag, err)
    print(mname, "worst rel err", max(worst.values()))


@pytest.mark.parametrize("mname", MODELS)
def test_logprob_proba_labels_after_estimate(golden_models, mname):
    """State semantics: after estimate_from_y the model is the observation-domain model of that SNR
    (SURVEY.md §3(D)); labels bit-exact, FP64 lp / proba."""
    _gpu_or_skip()
    fx = golden_models[mname]
    g = _model(fx)
    for tag in fx["cases"]:
        tag = str(tag)
        y, snr, N, A, n_bits, qtype, quantizer = case_args(fx, tag)
        g.estimate_from_y(y, snr, N, A, "all", n_bits, qtype, quantizer)
        np.testing.assert_array_equal(g._predict_cplx(y), fx[f"{tag}__labels"])
        # 1 bit with a general A: Cy = A C A^H has normalised entries at |rho| ~ 1 where the arcsine law
        # amplifies last-bit differences of the GEMM summation order ~1e7-fold; the reference itself is
        # reproducible only to ~1e-9 across BLAS builds there (tools/diag_lp.py), labels stay exact.
        tol = (1e-8, 1e-6) if tag.startswith("p2_b1") else (1e-10, 1e-8)
        prtol = 1e-7 if tol[1] < 1e-7 else 1e-5
        if g._dev.structure()[2] and n_bits == 1:
            # Fourier-domain path, 1 bit: the reference applies the arcsine law entry-wise to its dense
            # Cy = F^H diag(c) F + s2 I, whose entries along one circulant diagonal differ in the last
            # bits; near |rho| = 1 arcsin amplifies that (up to 3.8e-7 relative in lp at 20 dB, reproduced
            # by a NumPy restatement of the Fourier formulas); labels and h keep the normal bar
            tol, prtol = (1e-6, 1e-5), 1e-4
        np.testing.assert_allclose(g._estimate_weighted_log_prob(y), fx[f"{tag}__lp"], rtol=tol[0], atol=tol[1])
        np.testing.assert_allclose(g.predict_proba_cplx(y), fx[f"{tag}__proba"], rtol=prtol, atol=1e-13)


def test_prepare_tables_match_reference(golden_models):
    _gpu_or_skip()
    n = 0
    for mname in MODELS:
        fx = golden_models[mname]
        g = _model(fx)
        for tag in fx["cases"]:
            tag = str(tag)
            if f"{tag}__Cy" not in fx:
                continue
            y, snr, N, A, n_bits, qtype, quantizer = case_args(fx, tag)
            g.estimate_from_y(y[:2], snr, N, A, "all", n_bits, qtype, quantizer)
            t = g._dev.tables()
            assert rel_fro(t["Cy"][:2], fx[f"{tag}__Cy"]) < 1e-12
            sens = 1e4 if tag.startswith("p2_b1") else 1.0  # arcsine law at |rho| ~ 1, see above
            assert rel_fro(t["Cr"][:2], fx[f"{tag}__Cr"]) < 1e-12 * sens
            assert rel_fro(t["P"][:2], fx[f"{tag}__P"]) < 1e-10 * sens, (mname, tag)
            assert rel_fro(t["A_eff"][:2], fx[f"{tag}__A_eff"]) < 1e-12
            assert rel_fro(t["means_y"], fx[f"{tag}__means_y"]) < 1e-12
            W_ref = np.asarray(fx["covs_cplx"][:2]) @ np.conj(np.transpose(fx[f"{tag}__A_eff"], (0, 2, 1))) @ \
                fx[f"{tag}__Cr_inv"]
            assert rel_fro(t["W"][:2], W_ref) < 1e-9 * sens, (mname, tag)
            # mirrored sklearn state (:262-313)
            assert rel_fro(g.gm.means_, fx[f"{tag}__means_y"]) < 1e-12
            assert rel_fro(g.gm.precisions_cholesky_[:2], fx[f"{tag}__P"]) < 1e-10 * sens
            assert g.gm.n_features_in_ == A.shape[0]
            n += 1
    assert n >= 6


def test_channel_domain_predict_before_any_estimate(golden_models):
    """Before any estimate the reference's predict_proba_cplx uses the fit-state (channel-domain)
    model; the device path realises it as the prepare with A = I, sigma^2 = 0, n_bits = inf."""
    _gpu_or_skip()
    from oracle import qce_oracle as O
    fx = golden_models["fullmean"]
    g = _model(fx)
    h = fx["b1_5__h"]
    P = O.precision_cholesky(fx["covs_cplx"])
    ref = O.predict_proba(h, fx["means_cplx"], P, fx["weights"])
    np.testing.assert_allclose(g.predict_proba_cplx(h), ref, rtol=1e-7, atol=1e-13)
    np.testing.assert_array_equal(g._predict_cplx(h), O.predict(h, fx["means_cplx"], P, fx["weights"]))


def test_special_cases(golden_models):
    _gpu_or_skip()
    from quantized_channel_estimation_amd import Gmm_nbit, Gmm_quant
    fx = golden_models["full"]
    N = int(fx["N"])
    y = fx["b1_5__y"]
    g1 = Gmm_nbit.from_params(fx["means_cplx"][:1], fx["covs_cplx"][:1], np.array([1.0]))
    assert rel_fro(g1.estimate_from_y(y, 5, N, None, "all", 1), fx["k1__hest_all"]) < H_TOL
    g = _model(fx)
    assert rel_fro(g.estimate_from_y(y[:1], 5, N, None, "all", 1), fx["b1row__hest_all"]) < H_TOL
    # Gmm_quant twin (gmm_cplx_quant.py:190-267)
    gq = _model(fx, Gmm_quant)
    yq, snr, N, A, n_bits, qtype, quantizer = case_args(fx, "u2_5")
    assert rel_fro(gq.estimate_from_y(yq, snr, N, A, "all", n_bits, qtype, quantizer),
                   fx["quant_twin__hest_all"]) < H_TOL
    assert gq.eval_mode is True
    # picklable like the reference object sent through pool.starmap (Bussgang_GMM.py:282-287)
    g2 = pickle.loads(pickle.dumps(copy.deepcopy(g)))
    assert g2._dev is None
    assert rel_fro(g2.estimate_from_y(y, 5, N, None, "all", 1), fx["b1_5__hest_all"]) < H_TOL
    # empty batch
    assert g.estimate_from_y(y[:0], 5, N, None, "all", 1).shape == (0, N)


def _synthetic(K, N, B, seed, n_bits=1, snr=5.0, mean=False):
    from quantized_channel_estimation_amd import inputs
    means, covs, w = inputs.synthetic_model(K, N, seed=seed)
    rng = np.random.default_rng(seed + 1)
    if mean:
        means = 0.3 * inputs.crandn(K, N, rng=rng)
    h, _ = inputs.scm_generate(B, 1, N, rng, n_path=3)
    h = h[:, 0, :].astype(complex)
    thr = lab = None
    if n_bits not in (1, np.inf):
        thr, lab, _ = inputs.uniform_quantizer(snr, n_bits)
    y = inputs.get_observation_nbit(h, snr, None, n_bits, thr, lab, rng=rng)
    return means, covs, w, h, y, (thr, lab, None)


@pytest.mark.parametrize("K,N,B,n_bits,mean", [(64, 64, 3000, 1, False), (33, 48, 1000, 2, True),
                                               (16, 20, 257, np.inf, True), (128, 64, 2048, 1, False)])
def test_vs_oracle_larger(K, N, B, n_bits, mean):
    _gpu_or_skip()
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import Gmm_nbit
    means, covs, w, h, y, qz = _synthetic(K, N, B, 100 + K, n_bits, mean=mean)
    g = Gmm_nbit.from_params(means, covs, w)
    for mode in ("all", 1, 3, 0.9):
        hg = g.estimate_from_y(y, 5.0, N, None, mode, n_bits, "uniform", qz)
        ho = O.estimate(means, covs, w, y, 5.0, N, None, mode, n_bits, "uniform", qz)
        assert rel_fro(hg, ho) < H_TOL, (mode, rel_fro(hg, ho))
    t = O.prepare(means, covs, np.eye(N), 5.0, n_bits, "uniform", qz)
    np.testing.assert_array_equal(g._predict_cplx(y), O.predict(y, t["means_y"], t["P"], w))
    mse_g = np.mean(np.abs(g.estimate_from_y(y, 5.0, N, None, "all", n_bits, "uniform", qz) - h) ** 2)
    mse_o = np.mean(np.abs(O.estimate(means, covs, w, y, 5.0, N, None, "all", n_bits, "uniform", qz) - h) ** 2)
    assert abs(mse_g - mse_o) <= 1e-5 * mse_o


def test_k_shard_partials_combine_to_full():
    """Splitting the mixture into component shards and combining the partial (m, s, acc) gives the
    full 'all'-mode estimate (the K-shard data path)."""
    _gpu_or_skip()
    from quantized_channel_estimation_amd import Gmm_nbit
    from quantized_channel_estimation_amd.sharding import combine_partials_numpy
    from quantized_channel_estimation_amd import _lib
    K, N, B = 40, 32, 700
    means, covs, w, h, y, qz = _synthetic(K, N, B, 7, 1)
    full = Gmm_nbit.from_params(means, covs, w).estimate_from_y(y, 5.0, N, None, "all", 1)
    parts = []
    for lo, hi in [(0, 13), (13, 30), (30, 40)]:
        dm = _lib.DeviceModel(means[lo:hi], covs[lo:hi], w[lo:hi])
        dm.prepare(None, 5.0, 1.0)
        parts.append(dm.partial(y))
    hc = combine_partials_numpy(parts, N)
    assert rel_fro(hc, full) < 1e-6


def test_device_io_torch():
    _gpu_or_skip()
    import torch
    from quantized_channel_estimation_amd import _lib
    K, N, B = 32, 64, 4096
    means, covs, w, h, y, qz = _synthetic(K, N, B, 3, 1)
    dm = _lib.DeviceModel(means, covs, w)
    dm.prepare(None, 5.0, 1.0)
    host = dm.estimate(y)
    yd = torch.from_numpy(y).to("cuda")
    torch.cuda.synchronize()
    out = dm.estimate(yd)
    dm.synchronize()
    assert rel_fro(out.cpu().numpy(), host) == 0.0


@pytest.mark.parametrize("env", [{}, {"QCE_WORKGROUPS": "1"}, {"QCE_WORKGROUPS": "7"}, {"QCE_WORKGROUPS": "100"},
                                 {"QCE_WORKGROUPS": "5000"}, {"QCE_KERNEL": "f32"}, {"QCE_H2_NARROW": "1"}])
def test_all_mode_kernel_variants_vs_oracle(env, monkeypatch):
    """FP16 two-term split kernel (default) under different stream-K cuts (1 workgroup, uneven
    cuts, more workgroups than items), and the FP32-MFMA kernel, all agree with the FP64 oracle."""
    _gpu_or_skip()
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import Gmm_nbit
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    K, N, B = 64, 64, 3000
    means, covs, w, h, y, qz = _synthetic(K, N, B, 21, 1, mean=True)
    g = Gmm_nbit.from_params(means, covs, w)
    hg = g.estimate_from_y(y, 5.0, N, None, "all", 1)
    ho = O.estimate(means, covs, w, y, 5.0, N, None, "all", 1)
    assert rel_fro(hg, ho) < H_TOL, rel_fro(hg, ho)


@pytest.mark.parametrize("n_bits,snr", [(1, -10.0), (1, 20.0), (2, 5.0), (np.inf, 10.0)])
def test_inexact_observations_take_the_precise_path(n_bits, snr):
    """Observations that are not quantiser outputs (here: raw y declared as 1-bit / 2-bit) are not
    exact in fp16; the kernel detects that per wave and splits y too — results stay within tolerance."""
    _gpu_or_skip()
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import Gmm_nbit, inputs
    K, N, B = 48, 32, 1500
    means, covs, w = inputs.synthetic_model(K, N, seed=9)
    rng = np.random.default_rng(10)
    h, _ = inputs.scm_generate(B, 1, N, rng, n_path=3)
    y = h[:, 0, :].astype(complex) + 10 ** (-snr / 20) * inputs.crandn(B, N, rng=rng)  # unquantised
    qz = (None, None, None)
    if n_bits == 2:
        qz = inputs.uniform_quantizer(snr, 2)
    g = Gmm_nbit.from_params(means, covs, w)
    hg = g.estimate_from_y(y, snr, N, None, "all", n_bits, "uniform", qz)
    ho = O.estimate(means, covs, w, y, snr, N, None, "all", n_bits, "uniform", qz)
    assert rel_fro(hg, ho) < H_TOL, rel_fro(hg, ho)


def test_ragged_and_tiny_batches():
    _gpu_or_skip()
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import Gmm_nbit
    K, N = 20, 24
    means, covs, w, h, y, qz = _synthetic(K, N, 600, 33, 1)
    g = Gmm_nbit.from_params(means, covs, w)
    for B in (1, 2, 31, 255, 256, 257, 511, 600):
        hg = g.estimate_from_y(y[:B], 5.0, N, None, "all", 1)
        ho = O.estimate(means, covs, w, y[:B], 5.0, N, None, "all", 1)
        assert rel_fro(hg, ho) < H_TOL, (B, rel_fro(hg, ho))


# ---- large padded shapes (chunk-streamed kernel, qce_estimate_h2x.hip; FP64 lp + weighted selective modes)
@pytest.mark.parametrize("K,N,pilots,B,n_bits,mean", [
    (16, 128, 1, 700, 1, False),        # cfg4 geometry (N = 128), small K / B
    (7, 100, 1, 300, 2, True),          # padded N (100 -> 128), means, 2-bit uniform
    (5, 256, 1, 260, 1, False),         # cfg5 geometry (N = 256)
    (6, 64, 2, 300, 1, False),          # two pilots: M = 2N = 128 over N = 64
    (4, 128, 2, 140, 2, True),          # M = 256, N = 128
    (5, 200, 1, 150, np.inf, True),     # inexact observations at N = 256 padding (row-chunked path)
])
def test_large_shapes_vs_oracle(K, N, pilots, B, n_bits, mean):
    _gpu_or_skip()
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import Gmm_nbit, inputs
    means, covs, w = inputs.synthetic_model(K, N, seed=K + N)
    rng = np.random.default_rng(K * N)
    if mean:
        means = 0.3 * inputs.crandn(K, N, rng=rng)
    h, _ = inputs.scm_generate(B, 1, N, rng, n_path=3)
    h = h[:, 0, :].astype(complex)
    A = None if pilots == 1 else inputs.get_pilot_matrix(N, pilots, n_bits)
    qz = (None, None, None)
    if n_bits not in (1, np.inf):
        qz = inputs.uniform_quantizer(5.0, n_bits)
    y = inputs.get_observation_nbit(h, 5.0, A, n_bits, qz[0], qz[1], rng=rng)
    g = Gmm_nbit.from_params(means, covs, w)
    for mode in ("all", 1, 3, 0.9):
        hg = g.estimate_from_y(y, 5.0, N, A, mode, n_bits, "uniform", qz)
        ho = O.estimate(means, covs, w, y, 5.0, N, A, mode, n_bits, "uniform", qz)
        assert rel_fro(hg, ho) < H_TOL, (mode, rel_fro(hg, ho))
    t = O.prepare(means, covs, np.eye(N) if A is None else A, 5.0, n_bits, "uniform", qz)
    np.testing.assert_array_equal(g._predict_cplx(y), O.predict(y, t["means_y"], t["P"], w))


@pytest.mark.parametrize("ksplit", ["1", "2", "3", "7"])
def test_large_shape_k_splits_and_partials(ksplit, monkeypatch):
    """K splits of the large-shape kernel (merged by k_merge_splits) and its K-shard partial output."""
    _gpu_or_skip()
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import Gmm_nbit, _lib
    from quantized_channel_estimation_amd.sharding import combine_partials_numpy
    monkeypatch.setenv("QCE_KSPLIT", ksplit)
    K, N, B = 20, 128, 400
    means, covs, w, h, y, qz = _synthetic(K, N, B, 55, 1)
    ho = O.estimate(means, covs, w, y, 5.0, N, None, "all", 1)
    hg = Gmm_nbit.from_params(means, covs, w).estimate_from_y(y, 5.0, N, None, "all", 1)
    assert rel_fro(hg, ho) < H_TOL
    parts = []
    for lo, hi in [(0, 9), (9, 20)]:
        dm = _lib.DeviceModel(means[lo:hi], covs[lo:hi], w[lo:hi])
        dm.prepare(None, 5.0, 1.0)
        parts.append(dm.partial(y))
    assert rel_fro(combine_partials_numpy(parts, N), ho) < H_TOL


# ---- Fourier-domain path for (block-)circulant mixtures (qce_fft.hip)
def test_structure_detection_on_reference_fits(golden_models):
    """The reference's circulant / block-circulant fits (gmm_cplx_bussgang.py:104-133) are detected at
    model creation and prepared in the Fourier domain when A = I; a 'full' fit is not."""
    _gpu_or_skip()
    from quantized_channel_estimation_amd import _lib
    expect = {"circ": True, "bcirc": True, "full": False, "fullmean": False}
    for name, structured in expect.items():
        fx = golden_models[name]
        dm = _lib.DeviceModel(fx["means_cplx"], fx["covs_cplx"], fx["weights"])
        n1, n2, _ = dm.structure()
        assert (n1 > 0) == structured, (name, n1, n2)
        if structured:
            assert n1 * n2 == int(fx["N"])
            dm.prepare(None, 5.0, 1.0)
            assert dm.structure()[2] == 1
            A2 = np.kron(np.ones((2, 1)), np.eye(int(fx["N"])))  # two pilots: dense path
            dm.prepare(A2, 5.0, 1.0)
            assert dm.structure()[2] == 0


@pytest.mark.parametrize("K,N,blocks,B,n_bits,qtype,mean", [
    (128, 64, None, 2000, 3, "lloyd", False),   # cfg3 geometry: circulant, 3-bit Lloyd-Max
    (32, 256, (4, 64), 600, 2, "uniform", False),  # cfg5 geometry: block-circulant (4, 64), 2-bit
    (20, 32, (4, 8), 700, 1, "uniform", True),  # block-circulant with means
    (16, 16, None, 300, np.inf, "uniform", True),
])
def test_fourier_path_vs_oracle_and_dense(K, N, blocks, B, n_bits, qtype, mean, monkeypatch):
    _gpu_or_skip()
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import Gmm_nbit, inputs
    cov = "circulant" if blocks is None else "block-circulant"
    means, covs, w = inputs.synthetic_model(K, N, cov_type=cov, seed=K + N, blocks=blocks)
    rng = np.random.default_rng(N)
    if mean:
        means = 0.3 * inputs.crandn(K, N, rng=rng)
    h, _ = inputs.scm_generate(B, 1, N, rng, n_path=3)
    h = h[:, 0, :].astype(complex)
    qz = (None, None, None)
    if n_bits not in (1, np.inf):
        qz = inputs.get_quantizer([5.0], n_bits, qtype)[5.0]
    y = inputs.get_observation_nbit(h, 5.0, None, n_bits, qz[0], qz[1], rng=rng)
    g = Gmm_nbit.from_params(means, covs, w)
    res = {}
    for mode in ("all", 1, 3, 0.9):
        hg = g.estimate_from_y(y, 5.0, N, None, mode, n_bits, qtype, qz)
        assert g._dev.structure()[2] == 1
        ho = O.estimate(means, covs, w, y, 5.0, N, None, mode, n_bits, qtype, qz)
        # FP64 end to end, the selection weights included (k_select's FP64 weights); 1 bit: the arcsine-law
        # sensitivity of the dense restatement (see test_logprob_proba_labels_after_estimate)
        tol = 1e-9 if n_bits != 1 else 1e-7
        assert rel_fro(hg, ho) < tol, (mode, rel_fro(hg, ho))
        res[mode] = hg
    t = O.prepare(means, covs, np.eye(N), 5.0, n_bits, qtype, qz)
    g.estimate_from_y(y[:4], 5.0, N, None, "all", n_bits, qtype, qz)
    np.testing.assert_array_equal(g._dev.log_prob(y, want_lp=False, want_labels=True)[2],
                                  O.predict(y, t["means_y"], t["P"], w))
    # the dense kernels on the same model agree (QCE_FFT=0 keeps the prepare dense)
    monkeypatch.setenv("QCE_FFT", "0")
    gd = Gmm_nbit.from_params(means, covs, w)
    hd = gd.estimate_from_y(y, 5.0, N, None, "all", n_bits, qtype, qz)
    assert gd._dev.structure()[2] == 0
    assert rel_fro(hd, res["all"]) < H_TOL


def test_fourier_path_partials_combine():
    _gpu_or_skip()
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import _lib, inputs
    from quantized_channel_estimation_amd.sharding import combine_partials_numpy
    K, N, B = 24, 64, 500
    means, covs, w = inputs.synthetic_model(K, N, cov_type="circulant", seed=3)
    rng = np.random.default_rng(4)
    h, _ = inputs.scm_generate(B, 1, N, rng, n_path=3)
    y = inputs.get_observation_nbit(h[:, 0, :].astype(complex), 5.0, None, 1, rng=rng)
    parts = []
    for lo, hi in [(0, 10), (10, 24)]:
        dm = _lib.DeviceModel(means[lo:hi], covs[lo:hi], w[lo:hi])
        dm.prepare(None, 5.0, 1.0)
        assert dm.structure()[2] == 1
        parts.append(dm.partial(y))
    ho = O.estimate(means, covs, w, y, 5.0, N, None, "all", 1)
    assert rel_fro(combine_partials_numpy(parts, N), ho) < 1e-6


@pytest.mark.parametrize("K,N,blocks,B,n_bits,mean", [
    (40, 128, None, 333, 1, True),       # 1-D N=128: two waves split the bins; K padded to 48
    (7, 256, (2, 128), 101, 2, False),   # K < 16: one component block, mostly padding
    (130, 64, (8, 8), 777, 3, False),    # 2-D radix-8 x radix-8, K = 130 -> 144
    (33, 256, (4, 64), 64, np.inf, True),
])
def test_fourier_mfma_kernel_vs_lds_kernel(K, N, blocks, B, n_bits, mean, monkeypatch):
    """The MFMA Fourier kernel (qce_fft_mfma.hip, default) against the LDS-tiled FP64 kernel
    (qce_fft.hip, QCE_FFT_KERNEL=lds) and the oracle, 'all' mode and the K-shard partial."""
    _gpu_or_skip()
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import _lib, inputs
    from quantized_channel_estimation_amd.sharding import combine_partials_numpy
    cov = "circulant" if blocks is None else "block-circulant"
    means, covs, w = inputs.synthetic_model(K, N, cov_type=cov, seed=K, blocks=blocks)
    rng = np.random.default_rng(K + N)
    if mean:
        means = 0.3 * inputs.crandn(K, N, rng=rng)
    h, _ = inputs.scm_generate(B, 1, N, rng, n_path=3)
    qz = (None, None, None)
    qtype = "uniform"
    if n_bits not in (1, np.inf):
        qz = inputs.get_quantizer([5.0], n_bits, qtype)[5.0]
    y = inputs.get_observation_nbit(h[:, 0, :].astype(complex), 5.0, None, n_bits, qz[0], qz[1], rng=rng)
    out = {}
    for kern in ("mfma", "lds"):
        if kern == "lds":
            monkeypatch.setenv("QCE_FFT_KERNEL", "lds")
        dm = _lib.DeviceModel(means, covs, w)
        dm.prepare(None, 5.0, float(n_bits))
        assert dm.structure()[2] == 1
        out[kern] = (dm.estimate(y), combine_partials_numpy([dm.partial(y)], N),
                     combine_partials_numpy([dm.partial64(y)], N))
        dm.close()
    ho = O.estimate(means, covs, w, y, 5.0, N, None, "all", n_bits, qtype, qz)
    tol = 1e-9 if n_bits != 1 else 1e-7
    assert rel_fro(out["mfma"][0], ho) < tol
    assert rel_fro(out["mfma"][0], out["lds"][0]) < 1e-12
    assert rel_fro(out["mfma"][1], ho) < 1e-6  # qce_estimate_partial's acc is fp32 by its ABI
    for kern in ("mfma", "lds"):  # qce_estimate_partial_f64: the FP64 accumulator of the same kernels
        assert rel_fro(out[kern][2], ho) < tol, kern


@pytest.mark.parametrize("K,N,blocks,B,n_bits", [
    (128, 256, (4, 64), 1003, 2),   # cfg5 geometry: one chunk of 8 blocks, two per wave
    (200, 256, (16, 16), 517, 3),   # K = 200 -> 13 blocks: a second chunk of 5 (waves 1-3 one block each)
    (256, 128, (8, 16), 301, 2),    # two whole chunks (the Fourier path's largest K)
    (130, 128, None, 250, 2),       # 9 blocks: a second chunk of one block
    (7, 128, (2, 64), 33, 1),       # one padded block, three idle waves
    (64, 256, None, 100, 2),        # circulant 256: both register passes on one axis
    (40, 256, (2, 128), 90, 3),     # pass 1 = 3 bits of n2 + the n1 bit
    (48, 256, (64, 4), 77, 2),      # n2 = 4: pass 2 = both n2 bits + 2 low n1 bits, pass 1 n1 only (j != 0)
    # N = 64: k_fft_wreg (register transform, persistent one-wave tiles + cooperative tail)
    (128, 64, None, 3001, 3),       # cfg3 geometry, circulant: pass 1 = n2 bits 5, 4
    (64, 64, (2, 32), 500, 2),      # pass 1 = n2 bit 4 + the n1 bit
    (48, 64, (4, 16), 400, 2),      # pass 1 = both n1 bits, j = 0
    (40, 64, (16, 4), 300, 1),      # n2 = 4: pass 1 on n1 with j != 0, pass 2 mixes both axes
    (128, 64, None, 1, 3),          # one observation: a single ragged tile (descriptor-extent loads / stores)
    (128, 256, (4, 64), 5, 2),      # five observations on the N = 256 kernel
])
def test_fourier_chunk_kernel(K, N, blocks, B, n_bits, monkeypatch):
    """k_fft_chunk (zero-mean N = 128, 256: components split over the waves for lp / softmax, bins for the
    filter, two barriers per 128-component chunk) and k_fft_wreg (zero-mean N = 64) against the FP64 oracle and
    the kernels they replace (QCE_FFT_CHUNK=0: bin-split k_fft_mfma, LDS-transform k_fft_wave), 'all' mode and
    both K-shard partial accumulators."""
    _chunk_vs_oracle(K, N, blocks, B, n_bits, False, monkeypatch)


@pytest.mark.parametrize("K,N,blocks,B,n_bits", [
    (128, 256, (4, 64), 1003, 2),   # cfg5 geometry with means
    (200, 256, (16, 16), 517, 3),   # a second, partial chunk
    (256, 128, (8, 16), 301, 2),    # two whole chunks
    (130, 128, None, 250, np.inf),  # unquantised, a one-block second chunk
    (7, 128, (2, 64), 33, 1),       # one padded block, three idle waves
    (64, 256, None, 100, 2),        # circulant 256
    (48, 256, (64, 4), 77, 2),      # n2 = 4
    (128, 256, (4, 64), 5, 2),      # five observations
    # N = 64: k_fft_wreg<HM>
    (128, 64, None, 3001, 3),       # cfg3 geometry with means
    (64, 64, (2, 32), 500, 2),
    (40, 64, (16, 4), 300, 1),      # n2 = 4
    (128, 64, None, 1, 3),          # one observation
])
def test_fourier_chunk_kernel_means(K, N, blocks, B, n_bits, monkeypatch):
    """k_fft_chunk_hm (N = 128, 256 with means: the mean terms 2 Re(Y^* u) in the log-probabilities and
    sum_k gamma_k b_k in the filter, gmm_cplx_bussgang.py:256-264, :288) and k_fft_wreg<HM> (N = 64 with means)
    against the FP64 oracle and the kernels they replace (QCE_FFT_CHUNK=0: bin-split k_fft_mfma, LDS-transform
    k_fft_wave), 'all' mode and both K-shard partial accumulators."""
    _chunk_vs_oracle(K, N, blocks, B, n_bits, True, monkeypatch)


def _chunk_vs_oracle(K, N, blocks, B, n_bits, mean, monkeypatch):
    _gpu_or_skip()
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import _lib, inputs
    from quantized_channel_estimation_amd.sharding import combine_partials_numpy
    cov = "circulant" if blocks is None else "block-circulant"
    means, covs, w = inputs.synthetic_model(K, N, cov_type=cov, seed=K + 1, blocks=blocks)
    rng = np.random.default_rng(K * N)
    means = 0.3 * inputs.crandn(K, N, rng=rng) if mean else np.zeros_like(means)
    h, _ = inputs.scm_generate(B, 1, N, rng, n_path=3)
    qz = (None, None, None)
    if n_bits not in (1, np.inf):
        qz = inputs.get_quantizer([5.0], n_bits, "uniform")[5.0]
    y = inputs.get_observation_nbit(h[:, 0, :].astype(complex), 5.0, None, n_bits, qz[0], qz[1], rng=rng)
    out = {}
    for chunk in ("1", "0"):
        monkeypatch.setenv("QCE_FFT_CHUNK", chunk)
        dm = _lib.DeviceModel(means, covs, w)
        dm.prepare(None, 5.0, float(n_bits))
        assert dm.structure()[2] == 1
        out[chunk] = (dm.estimate(y), combine_partials_numpy([dm.partial(y)], N),
                      combine_partials_numpy([dm.partial64(y)], N))
        dm.close()
    ho = O.estimate(means, covs, w, y, 5.0, N, None, "all", n_bits, "uniform", qz)
    tol = 1e-9 if n_bits != 1 else 1e-7
    assert rel_fro(out["1"][0], ho) < tol, rel_fro(out["1"][0], ho)
    assert rel_fro(out["1"][0], out["0"][0]) < 1e-12
    assert rel_fro(out["1"][1], ho) < 1e-6  # qce_estimate_partial's acc is fp32 by its ABI
    assert rel_fro(out["1"][2], ho) < tol


@pytest.mark.parametrize("K,N,blocks,B,n_bits,qtype,mean", [
    (128, 64, None, 70013, 3, "lloyd", False),   # cfg3 geometry: two whole rounds of tiles + a ragged tail
    (64, 64, (8, 8), 70013, 1, "uniform", False),  # 2-D transform through the same phases
    (16, 16, (4, 4), 40013, 2, "uniform", False),
    (32, 32, None, 20013, np.inf, "uniform", True),  # with means: every tile one wave, persistent loop
    (128, 64, None, 40013, 3, "lloyd", True),  # cfg3 with means: k_fft_wreg<HM>, one workgroup per CU
])
def test_fourier_wave_kernel_persistent_phases(K, N, blocks, B, n_bits, qtype, mean, monkeypatch):
    """k_fft_wave (N <= 64) at batches large enough for its main phase: one wave per 16-row tile over
    whole rounds of the persistent grid, with the next tile's y prefetched behind the current one, then
    the remainder worked cooperatively by the four waves of a workgroup (zero-mean models).  Small-batch
    tests reach only the cooperative phase.  One launch (QCE_HOST_PIPELINE=0); rows from the first
    round, the main/tail boundary and the ragged end are checked against the FP64 oracle, and the first
    rows against the same rows estimated alone (cooperative phase), to FP64 rounding."""
    _gpu_or_skip()
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import Gmm_nbit, inputs
    monkeypatch.setenv("QCE_HOST_PIPELINE", "0")
    cov = "circulant" if blocks is None else "block-circulant"
    means, covs, w = inputs.synthetic_model(K, N, cov_type=cov, seed=K + N, blocks=blocks)
    rng = np.random.default_rng(B)
    if mean:
        means = 0.3 * inputs.crandn(K, N, rng=rng)
    h = inputs.crandn(B, N, rng=rng)
    qz = (None, None, None)
    if n_bits not in (1, np.inf):
        qz = inputs.get_quantizer([5.0], n_bits, qtype)[5.0]
    y = inputs.get_observation_nbit(h, 5.0, None, n_bits, qz[0], qz[1], rng=rng)
    g = Gmm_nbit.from_params(means, covs, w)
    hg = g.estimate_from_y(y, 5.0, N, None, "all", n_bits, qtype, qz)
    assert g._dev.structure()[2] == 1
    assert hg.shape == (B, N) and np.isfinite(hg).all()
    tol = 1e-9 if n_bits != 1 else 1e-7
    ntiles = (B + 15) // 16
    per_round = 1024 if (N == 64 and mean) else 2048  # 256 CUs x 2 workgroups (1 for k_fft_wreg<HM>) x 4 waves
    edge = (ntiles // per_round) * per_round * 16  # main/tail boundary
    for lo, hi in ((0, 200), (max(edge - 100, 0), edge + 100), (B - 200, B)):
        ho = O.estimate(means, covs, w, y[lo:hi], 5.0, N, None, "all", n_bits, qtype, qz)
        assert rel_fro(hg[lo:hi], ho) < tol, (lo, hi, rel_fro(hg[lo:hi], ho))
    alone = g.estimate_from_y(y[:300], 5.0, N, None, "all", n_bits, qtype, qz)
    assert rel_fro(hg[:300], alone) < 1e-12
