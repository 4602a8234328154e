"""BASELINE.json configurations at their own model sizes (full K), through the C-ABI, against the
FP64 oracle: cfg4 (K=256, N=128, 'full', 1 bit) and cfg5 (K=128, N=256, block-circulant (4, 64),
2-bit uniform) — every mode, the Fourier path and the dense path, and the K-shard partials that
the multi-GPU split all-reduces.  Batches are reduced (the oracle's 'all' mode materialises
B x K x N filter outputs); the full batch sizes run in bench.py with parity on 512 samples."""
import numpy as np
import pytest

from conftest import rel_fro

pytestmark = pytest.mark.gpu

F64_TOL = 1e-9
H_TOL = 1e-5


def _inputs(K, N, B, cov, blocks, n_bits, seed):
    from quantized_channel_estimation_amd import inputs
    means, covs, w = inputs.synthetic_model(K, N, cov_type=cov, blocks=blocks)
    rng = np.random.default_rng(seed)
    h, _ = inputs.scm_generate(B, 1, N, rng, n_path=3)
    h = h[:, 0, :].astype(complex)
    qz = (None, None, None)
    if n_bits not in (1, np.inf):
        qz = inputs.get_quantizer([5.0], n_bits, "uniform")[5.0]
    y = inputs.get_observation_nbit(h, 5.0, None, n_bits, qz[0], qz[1], rng=rng)
    return means, covs, w, h, y, qz


def _shard_combine(means, covs, w, y, n_bits, cuts):
    from quantized_channel_estimation_amd import _lib
    from quantized_channel_estimation_amd.sharding import combine_packed_numpy
    models = []
    for lo, hi in cuts:
        d = _lib.DeviceModel(means[lo:hi], covs[lo:hi], w[lo:hi])
        d.prepare(None, 5.0, float(n_bits))
        models.append(d)
    shift = max(float(np.max(d.cconst())) for d in models)
    return combine_packed_numpy([d.partial_shifted(y, shift) for d in models])


def test_cfg4_all_modes_and_kshard():
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import Gmm_nbit
    K, N, B = 256, 128, 1024
    means, covs, w, h, y, qz = _inputs(K, N, B, "full", None, 1, 4004)
    g = Gmm_nbit.from_params(means, covs, w)
    for mode, tol in (("all", F64_TOL), (1, F64_TOL), (3, F64_TOL), (0.9, F64_TOL)):
        hg = g.estimate_from_y(y, 5.0, N, None, mode, 1)
        ho = O.estimate(means, covs, w, y, 5.0, N, None, mode, 1)
        assert rel_fro(hg, ho) < tol, (mode, rel_fro(hg, ho))
        if mode == "all":
            h_all = ho
    t = O.prepare(means, covs, np.eye(N), 5.0, 1)
    np.testing.assert_array_equal(g._predict_cplx(y), O.predict(y, t["means_y"], t["P"], w))
    # K shards of the north-star split (2 and 8 ranks' worth of components)
    for cuts in ([(0, 128), (128, 256)], [(32 * r, 32 * r + 32) for r in range(8)]):
        assert rel_fro(_shard_combine(means, covs, w, y, 1, cuts), h_all) < F64_TOL


@pytest.mark.parametrize("fft", ["1", "0"])
def test_cfg5_fourier_and_dense(fft, monkeypatch):
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import Gmm_nbit
    monkeypatch.setenv("QCE_FFT", fft)
    K, N, B = 128, 256, 256
    means, covs, w, h, y, qz = _inputs(K, N, B, "block-circulant", (4, 64), 2, 5005)
    g = Gmm_nbit.from_params(means, covs, w)
    for mode in ("all", 1, 3, 0.9):
        hg = g.estimate_from_y(y, 5.0, N, None, mode, 2, "uniform", qz)
        assert g._dev.structure()[2] == (1 if fft == "1" else 0)
        ho = O.estimate(means, covs, w, y, 5.0, N, None, mode, 2, "uniform", qz)
        # FP64 throughout on both paths: Fourier (selection weights included) and dense N = 256 ('all' on the
        # two-pass FP64 kernels k_lp_f64 + k_wsum_f64)
        assert rel_fro(hg, ho) < F64_TOL, (fft, mode, rel_fro(hg, ho))
    h_all = O.estimate(means, covs, w, y, 5.0, N, None, "all", 2, "uniform", qz)
    assert rel_fro(_shard_combine(means, covs, w, y, 2, [(0, 64), (64, 128)]), h_all) < F64_TOL


@pytest.mark.parametrize("n_pilots,N,K,n_bits,mean", [(4, 64, 32, 1, False), (4, 64, 24, 3, True),
                                                     (2, 128, 16, 1, False), (1, 256, 12, np.inf, True),
                                                     (8, 32, 20, 2, False)])
def test_dense_padded_256_fp64(n_pilots, N, K, n_bits, mean):
    """Dense shapes whose padded observation or channel dimension is 256 (M = n_pilots N with the scripts'
    pilot matrix, utils.py:337-367; or N = 256): every mode and the K-shard partials in FP64 at 1e-9."""
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import Gmm_nbit, inputs, _lib
    from quantized_channel_estimation_amd.sharding import UNDERFLOW_S, combine_packed_numpy, combine_partials_numpy
    rng = np.random.default_rng(600 + N + K)
    means, covs, w = inputs.synthetic_model(K, N, seed=7 + K)
    if mean:
        means = 0.3 * (rng.standard_normal((K, N)) + 1j * rng.standard_normal((K, N)))
    A = inputs.get_pilot_matrix(N, n_pilots, n_bits)
    B = 300
    h, _ = inputs.scm_generate(B, 1, N, rng, n_path=3)
    h = h[:, 0, :].astype(complex)
    qtype = "uniform"
    qz = (None, None, None)
    if n_bits not in (1, np.inf):
        qz = inputs.get_quantizer([5.0], n_bits, qtype)[5.0]
    y = inputs.get_observation_nbit(h, 5.0, A, n_bits, qz[0], qz[1], rng=rng)
    g = Gmm_nbit.from_params(means, covs, w)
    for mode in ("all", 1, 3, 0.9):
        hg = g.estimate_from_y(y, 5.0, N, A, mode, n_bits, qtype, qz)
        ho = O.estimate(means, covs, w, y, 5.0, N, A, mode, n_bits, qtype, qz)
        # 1 bit with a non-identity A: the arcsine-law sensitivity documented in test_gpu_parity (1e-8 there)
        tol = 1e-7 if (n_bits == 1 and n_pilots > 1) else F64_TOL
        assert rel_fro(hg, ho) < tol, (mode, rel_fro(hg, ho))
        if mode == "all":
            h_all = hg
    # K-shard partials of the same path: (m, s, acc) in FP64, and the shifted packed rows
    cuts = [(0, K // 2), (K // 2, K)]
    models = []
    for lo, hi in cuts:
        d = _lib.DeviceModel(means[lo:hi], covs[lo:hi], w[lo:hi])
        d.prepare(A, 5.0, float(n_bits), _lib.QUANT_UNIFORM)
        models.append(d)
    shift = max(d.cconst_max() for d in models)
    packed = [d.partial_shifted(y, shift) for d in models]
    # rows whose shifted sum leaves the normal range are the sharding layer's exact-recombination rows
    # (unquantised y with means: quad forms of several hundred); the others must match
    ok = np.sum([p[:, 0] for p in packed], axis=0) >= UNDERFLOW_S
    assert ok.mean() > 0.2
    with np.errstate(invalid="ignore", divide="ignore"):
        hp = combine_packed_numpy(packed)
    assert rel_fro(hp[ok], h_all[ok]) < 1e-12
    hm = combine_partials_numpy([tuple(d.partial64(y)) for d in models], N)
    assert rel_fro(hm, h_all) < 1e-12


@pytest.mark.gpu
def test_bench_kshard_two_ranks_gloo_one_gpu():
    """The multi-GPU bench path end to end: `bench.py --gpus 2` launches two ranks (here sharing the one
    GPU, collectives over gloo), each estimates its half of the K components with the FP64 partial kernel,
    the shifted partials are reduce-scattered per batch chunk, and the combined estimate matches the FP64
    oracle (the driver runs the same path over RCCL on 2/4/8 GPUs)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--batch", "4096", "--steps", "2", "--warmup", "1", "--cpu-seconds", "0", "--no-extras"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    d = json.loads(line[-1])
    assert d["world_size"] == 2 and d["config"]["shard"] == "k" and d["dtype"] == "f64"
    assert d["parity"]["rel_fro"] < 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("K", [300, 1000])
def test_wide_k_all_modes(K):
    """K beyond one wave's 256 components: 'all', argmax, top-3, cumulative-p 0.9, predict_proba and the labels
    (k_select_wide: the row in LDS, a bitonic sort of (proba, index)) against the FP64 oracle
    (gmm_cplx_bussgang.py:197-243, :335-367)."""
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import _lib, inputs
    means, covs, w = inputs.synthetic_model(K, 16, seed=9)
    rng = np.random.default_rng(9)
    y = (np.sign(rng.standard_normal((40, 16))) + 1j * np.sign(rng.standard_normal((40, 16)))) / np.sqrt(2)
    dm = _lib.DeviceModel(means, covs, w)
    dm.prepare(None, 5.0, 1.0)
    for mode, (cm, param) in (("all", (_lib.MODE_ALL, 0.0)), (1, (_lib.MODE_TOPN, 1.0)), (3, (_lib.MODE_TOPN, 3.0)),
                              (0.9, (_lib.MODE_CUMP, 0.9))):
        h = dm.estimate(y, cm, param)
        assert rel_fro(h, O.estimate(means, covs, w, y, 5.0, 16, None, mode, 1)) < 1e-9, mode
    t = O.prepare(means, covs, np.eye(16), 5.0, 1)
    lp, pr, lab = dm.log_prob(y, want_lp=True, want_proba=True, want_labels=True)
    np.testing.assert_array_equal(lab, O.predict(y, t["means_y"], t["P"], w))
    np.testing.assert_allclose(pr, O.predict_proba(y, t["means_y"], t["P"], w), rtol=1e-9, atol=1e-15)
    dm.close()


@pytest.mark.parametrize("N,pilots,K,with_mean", [(320, 1, 6, False), (288, 1, 5, True), (136, 2, 4, False)])
def test_wide_dimensions_all_modes(N, pilots, K, with_mean):
    """Channel / observation dimensions beyond 256 (the GEMM-based FP64 path, qce_big.hip): N = 320 and 288 (with
    means) with A = I, and N = 136 with 2 pilots (M = 272, a general A): 'all', argmax, top-3, cumulative-p 0.9 and
    predict_proba against the FP64 oracle at 1e-9; the reference runs any N (gmm_cplx_bussgang.py:197-243)."""
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import _lib, inputs
    means, covs, w = inputs.synthetic_model(K, N, seed=3)
    rng = np.random.default_rng(4)
    if with_mean:
        means = 0.3 * (rng.standard_normal((K, N)) + 1j * rng.standard_normal((K, N)))
    M = N * pilots
    A = None if pilots == 1 else np.kron(np.exp(2j * np.pi * rng.random((pilots, 1))), np.eye(N)) / np.sqrt(pilots)
    y = (np.sign(rng.standard_normal((48, M))) + 1j * np.sign(rng.standard_normal((48, M)))) / np.sqrt(2)
    dm = _lib.DeviceModel(means, covs, w)
    dm.prepare(A, 5.0, 1.0)
    Ao = np.eye(N) if A is None else A
    tol = 1e-9 if pilots == 1 else 1e-6  # 1 bit with a general A: the arcsine law's documented sensitivity
    for mode, (cm, param) in (("all", (_lib.MODE_ALL, 0.0)), (1, (_lib.MODE_TOPN, 1.0)), (3, (_lib.MODE_TOPN, 3.0)),
                              (0.9, (_lib.MODE_CUMP, 0.9))):
        h = dm.estimate(y, cm, param)
        ho = O.estimate(means, covs, w, y, 5.0, N, Ao, mode, 1)
        assert rel_fro(h, ho) < tol, (mode, rel_fro(h, ho))
    t = O.prepare(means, covs, Ao, 5.0, 1)
    _, pr, lab = dm.log_prob(y, want_lp=False, want_proba=True, want_labels=True)
    np.testing.assert_array_equal(lab, O.predict(y, t["means_y"], t["P"], w))
    np.testing.assert_allclose(pr, O.predict_proba(y, t["means_y"], t["P"], w), rtol=1e-6, atol=1e-12)
    # the K-shard partial of this path recombines to the same estimate
    m_, s_, a_ = dm.partial64(y)
    from quantized_channel_estimation_amd.sharding import combine_partials_numpy
    hp = combine_partials_numpy([(m_, s_, a_)], N)
    assert rel_fro(hp, O.estimate(means, covs, w, y, 5.0, N, Ao, "all", 1)) < tol
    dm.close()
    import ctypes
    h = ctypes.c_void_p()
    one = np.ones(2)
    with pytest.raises(NotImplementedError):  # beyond QCE_BIG_MAX: refused before any upload
        _lib.check(_lib.load().qce_model_create(1, 4097, None, _lib.ptr(one), _lib.ptr(one), 0, ctypes.byref(h)))


def test_wide_dimensions_all_mode_beyond_select_k():
    """'all' mode on the GEMM path (N > 256) with K beyond the selection kernels' K (4096) takes its
    responsibilities from a K-unbounded row kernel.  Mixture of 5 distinct components, each repeated 820 times
    (K = 4100) with its weight split evenly: the estimate equals the 5-component mixture's (FP64 oracle, 1e-9)."""
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import _lib, inputs
    N, Kd, rep = 264, 5, 820
    means, covs, w = inputs.synthetic_model(Kd, N, seed=5)
    assert Kd * rep > 4096  # qce_select_max_k (k_select_wide)
    rng = np.random.default_rng(6)
    y = (np.sign(rng.standard_normal((32, N))) + 1j * np.sign(rng.standard_normal((32, N)))) / np.sqrt(2)
    dm = _lib.DeviceModel(np.repeat(means, rep, axis=0), np.repeat(covs, rep, axis=0), np.repeat(w / rep, rep))
    dm.prepare(None, 5.0, 1.0)
    h = dm.estimate(y, _lib.MODE_ALL, 0.0)
    ho = O.estimate(means, covs, w, y, 5.0, N, None, "all", 1)
    assert rel_fro(h, ho) < 1e-9, rel_fro(h, ho)
    dm.close()
