"""Host numpy I/O of qce_estimate (the drop-in path of Gmm_nbit.estimate_from_y,
gmm_cplx_bussgang.py:166-243): batches large enough to split run chunked over copy-in / compute / copy-out streams,
DMA'ed straight from the caller's y (registered for the call) into the result array (page-locked, from the
library's result pool, or registered) -- or, with QCE_HOST_DIRECT=0 or memory that cannot be registered, through
the staged pipeline (host copies into pinned slots).  Every sample is independent, so the result equals the one-shot host path
(QCE_HOST_PIPELINE=0) and device-resident I/O: bit-identical for the Fourier path and the selective
modes; the dense 'all' kernel balances its launch by splitting K over workgroups (stream-K) with a split
chosen from the launch's batch size, so a chunk can sum the components in another order -- there the bar
is FP64 rounding (1e-12 relative Frobenius).  The ragged last chunk is checked against the oracle."""
import numpy as np
import pytest

from conftest import rel_fro

pytestmark = pytest.mark.gpu


def _gpu_or_skip():
    from quantized_channel_estimation_amd import _lib
    if _lib.device_count() == 0:
        pytest.fail("no GPU visible for a gpu-marked test")


@pytest.mark.parametrize("K,N,B,cov,mode", [
    (16, 32, 20001, "full", "all"),        # 5 chunks of 4096 rows + a ragged tail
    (8, 64, 9000, "full", 1),              # argmax mode through the pipeline
    (12, 64, 12345, "circulant", "all"),   # Fourier path
])
def test_host_pipeline_bit_identical(K, N, B, cov, mode, monkeypatch):
    _gpu_or_skip()
    import torch
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import _lib, inputs
    means, covs, w = inputs.synthetic_model(K, N, cov_type=cov, seed=K + N)
    rng = np.random.default_rng(B)
    h, _ = inputs.scm_generate(B, 1, N, rng, n_path=3)
    y = inputs.get_observation_nbit(h[:, 0, :].astype(complex), 5.0, None, 1, rng=rng)
    md = {"all": _lib.MODE_ALL, 1: _lib.MODE_TOPN}[mode]
    par = 0.0 if mode == "all" else 1.0
    dm = _lib.DeviceModel(means, covs, w)
    dm.prepare(None, 5.0, 1.0)
    assert dm.structure()[2] == (1 if cov == "circulant" else 0)
    h_pipe = dm.estimate(y, md, par)                                        # direct DMA, pooled pinned result
    h_reg = dm.estimate(y, md, par, out=np.empty((B, N), dtype=complex))    # direct DMA, result registered
    monkeypatch.setenv("QCE_HOST_DIRECT", "0")
    h_staged = dm.estimate(y, md, par)                                      # staged pipeline
    monkeypatch.delenv("QCE_HOST_DIRECT")
    h_dev = dm.estimate(torch.from_numpy(y).to("cuda"), md, par).cpu().numpy()
    monkeypatch.setenv("QCE_HOST_PIPELINE", "0")
    h_one = dm.estimate(y, md, par)
    for hx in (h_pipe, h_reg, h_staged):
        if mode == "all" and cov == "full":
            assert rel_fro(hx, h_one) < 1e-12 and rel_fro(hx, h_dev) < 1e-12
        else:
            np.testing.assert_array_equal(hx, h_one)
            np.testing.assert_array_equal(hx, h_dev)
    sl = slice(B - 300, B)  # the ragged last chunk against the FP64 oracle
    ho = O.estimate(means, covs, w, y[sl], 5.0, N, None, mode, 1)
    assert rel_fro(h_pipe[sl], ho) < 1e-7
    dm.close()


def test_pinned_result_pool_reuse_and_isolation():
    """The drop-in results come from a pool of page-locked blocks: a dropped result's block serves the next call,
    a live result is never overwritten by a later call, and the arrays behave as ordinary numpy arrays."""
    _gpu_or_skip()
    import gc
    from quantized_channel_estimation_amd import _lib, inputs
    K, N, B = 8, 64, 40000
    means, covs, w = inputs.synthetic_model(K, N, seed=9)
    rng = np.random.default_rng(9)
    y1 = (np.sign(rng.standard_normal((B, N))) + 1j * np.sign(rng.standard_normal((B, N)))) / np.sqrt(2)
    y2 = -y1
    dm = _lib.DeviceModel(means, covs, w)
    dm.prepare(None, 5.0, 1.0)
    h1 = dm.estimate(y1)
    assert isinstance(h1.base, _lib._PinnedArrayBase)
    keep = h1.copy()
    h2 = dm.estimate(y2)  # h1 is alive: a second block
    assert h2.base.blk.ptr != h1.base.blk.ptr
    np.testing.assert_array_equal(h1, keep)
    np.testing.assert_allclose(h2, -h1, rtol=0, atol=1e-12)  # zero-mean model: h(-y) = -h(y)
    p1 = h1.base.blk.ptr
    del h1
    gc.collect()
    h3 = dm.estimate(y1)  # reuses the dropped block
    assert h3.base.blk.ptr == p1
    assert rel_fro(h3, keep) < 1e-13
    dm.close()
