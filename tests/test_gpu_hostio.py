"""Host numpy I/O of qce_estimate (the drop-in path of Gmm_nbit.estimate_from_y,
gmm_cplx_bussgang.py:166-243): batches large enough to split run through the chunked pinned pipeline
(copy-in / compute / copy-out streams).  Every sample is independent, so the result equals the one-shot host path
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
    h_pipe = dm.estimate(y, md, par)
    h_dev = dm.estimate(torch.from_numpy(y).to("cuda"), md, par).cpu().numpy()
    monkeypatch.setenv("QCE_HOST_PIPELINE", "0")
    h_one = dm.estimate(y, md, par)
    if mode == "all" and cov == "full":
        assert rel_fro(h_pipe, h_one) < 1e-12 and rel_fro(h_pipe, h_dev) < 1e-12
    else:
        np.testing.assert_array_equal(h_pipe, h_one)
        np.testing.assert_array_equal(h_pipe, h_dev)
    sl = slice(B - 300, B)  # the ragged last chunk against the FP64 oracle
    ho = O.estimate(means, covs, w, y[sl], 5.0, N, None, mode, 1)
    assert rel_fro(h_pipe[sl], ho) < 1e-7
    dm.close()
