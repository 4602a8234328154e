"""One rank of a multi-GPU K-shard step, rehearsed on the one GPU of the box, and the lifecycle of the library's
K-shard objects.

* QCE_KSHARD_EMULATE_WORLD="W:R" on a world-1 RCCL communicator lays the step's rows out as rank R of W ranks: the
  shard computes its components over all B rows, reduce-scatters and finalises only its own B / W rows.  Those rows
  must equal the single-GPU estimate of the same mixture (the rank's share of the per-rank work is then the real one,
  only the wire time is missing).
* A process that runs a K-shard step over RCCL and exits without closing anything must exit with status 0 (the
  atexit hook of _lib closes every live handle while the runtimes are up).
* KShard.estimate with the default stream orders the reuse of a dropped step's tensors behind the step's
  communication-stream work.

Reference: Bussgang_GMM.py:29-32, :284-287 (the SNR process pool the K-shard replaces); gmm_cplx_bussgang.py:220-228."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, case_args, load_model, rel_fro

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl1():
    from quantized_channel_estimation_amd import _lib
    from quantized_channel_estimation_amd.sharding import make_comm
    if _lib.device_count() == 0:
        pytest.fail("no GPU visible for a gpu-marked test")
    comm = make_comm(0, 1, 0, kind="rccl")
    yield comm
    comm.close()


def _metric_batch(K, N, B, seed=77):
    from quantized_channel_estimation_amd import inputs
    means, covs, w = inputs.synthetic_model(K, N)
    rng = np.random.default_rng(seed)
    hp, _ = inputs.scm_generate(1024, 1, N, rng, n_path=3)
    h = hp[:, 0, :].astype(complex)[rng.integers(0, 1024, size=B)]
    y = np.ascontiguousarray(inputs.get_observation_nbit(h, 5.0, None, 1, rng=rng), dtype=np.complex128)
    return means, covs, w, y


@pytest.mark.parametrize("world,rank,chunks,agree_first", [(8, 0, 1, 0), (8, 5, 1, 0), (4, 3, 2, 0), (8, 7, 1, 0),
                                                            (8, 3, 1, 1), (4, 1, 2, 1)])
def test_emulated_world_rank_rows_equal_single_gpu(rccl1, monkeypatch, world, rank, chunks, agree_first):
    """Rank `rank` of an emulated `world`-GPU step (K = 16 components per rank at the metric's N = 64, B = 20001 so
    the last chunk is ragged): the rows returned are exactly the rank's reduce-scatter slice and equal the single-GPU
    estimate of the same mixture to 1e-12.  agree_first = 1: the shift MAX before the partial kernel, rows written
    shifted by the agreed M* and summed unscaled (QCE_KSHARD_AGREE_FIRST, the A/B alternative to the scaling pass)."""
    import torch
    from quantized_channel_estimation_amd import _lib
    from quantized_channel_estimation_amd.sharding import ComponentShardEstimator, chunk_bounds
    monkeypatch.setenv("QCE_KSHARD_EMULATE_WORLD", f"{world}:{rank}")
    monkeypatch.setenv("QCE_KSHARD_AGREE_FIRST", str(agree_first))
    K, N, B = 16, 64, 20001
    means, covs, w, y = _metric_batch(K, N, B)
    est = ComponentShardEstimator(means, covs, w, 0, 1, device=0, comm=rccl1, double_buffer=True)
    assert (est.native.layout_world, est.native.layout_rank) == (world, rank)
    single = _lib.DeviceModel(means, covs, w, device=0)
    yd = torch.from_numpy(y).cuda()
    for snr in (5.0, -5.0):
        est.prepare(None, snr, 1)
        single.prepare(None, snr, 1)
        rows, h = est.estimate(yd, chunks=chunks, scatter=True)
        r = rows.cpu().numpy()
        want = []
        for lo, hi in chunk_bounds(B, chunks, world, True):
            q = -(-(hi - lo) // world)
            want.extend(range(lo + rank * q, min(hi, lo + (rank + 1) * q)))
        assert r.tolist() == want
        hs = single.estimate(y[r])
        assert rel_fro(h.cpu().numpy(), hs) < 1e-12, (world, rank, snr)
    with pytest.raises(NotImplementedError):
        est.estimate(yd, mode=_lib.MODE_TOPN, param=1.0)
    est.close()
    single.close()


def test_emulated_world_underflow_rows_recombined(rccl1, monkeypatch):
    """The exact recombination of flagged rows (finish()) under the emulated layout: QCE_KSHARD_GLOBAL_BIAS zeroes
    every row through the PreMulSum, only the rank's B / W rows are flagged, and they come back exact."""
    import torch
    from quantized_channel_estimation_amd import _lib
    from quantized_channel_estimation_amd.sharding import ComponentShardEstimator
    monkeypatch.setenv("QCE_KSHARD_EMULATE_WORLD", "8:2")
    fx = load_model("full")
    y, snr, N, A, n_bits, qtype, quantizer = case_args(fx, "b1_5")
    est = ComponentShardEstimator(fx["means_cplx"], fx["covs_cplx"], fx["weights"], 0, 1, device=0, comm=rccl1)
    single = _lib.DeviceModel(fx["means_cplx"], fx["covs_cplx"], fx["weights"], device=0)
    est.prepare(None, snr, 1)
    single.prepare(None, snr, 1)
    yd = torch.from_numpy(np.ascontiguousarray(y)).cuda()
    monkeypatch.setenv("QCE_KSHARD_GLOBAL_BIAS", "2000")
    rows, h = est.estimate(yd, chunks=1, scatter=True)
    r = rows.cpu().numpy()
    assert est.native.flags()[0] == r.size > 0
    assert rel_fro(h.cpu().numpy(), single.estimate(np.ascontiguousarray(y))[r]) < 1e-12
    est.close()
    single.close()


def test_default_stream_reuse_after_lagging_comm_stream(rccl1, monkeypatch):
    """KShard.estimate without a stream, the communication stream held 3 ms per step, a fresh y per
    step and torch allocations between the steps (which would land on a dropped step's y / h if the allocator could
    reuse them before the step's collectives ran): every step's h equals the single-GPU result."""
    import torch
    from quantized_channel_estimation_amd import _lib
    from quantized_channel_estimation_amd.sharding import make_comm  # noqa: F401
    fx = load_model("fullmean")
    y, _, N, A, n_bits, qtype, quantizer = case_args(fx, "b1_5")
    dev = _lib.DeviceModel(fx["means_cplx"], fx["covs_cplx"], fx["weights"], device=0)
    ks = _lib.KShard(dev, rccl1, dev.K)
    single = _lib.DeviceModel(fx["means_cplx"], fx["covs_cplx"], fx["weights"], device=0)
    ks.prepare(None, 5.0, 1)
    single.prepare(None, 5.0, 1)
    ref = single.estimate(np.ascontiguousarray(y))
    monkeypatch.setenv("QCE_KSHARD_CS_DELAY_US", "3000")
    outs = []
    rng = np.random.default_rng(3)
    for i in range(5):
        yd = torch.from_numpy(np.ascontiguousarray(y)).cuda()
        rows, h = ks.estimate(yd, chunks=1, scatter=False)
        outs.append(h)
        del yd
        junk = [torch.from_numpy(rng.standard_normal(y.shape) + 0j).cuda() for _ in range(3)]  # reuse pressure
        del junk
    ks.finish()
    torch.cuda.synchronize()
    for i, h in enumerate(outs):
        assert rel_fro(h.cpu().numpy(), ref) < 1e-12, i
    ks.close()
    dev.close()
    single.close()


@pytest.mark.parametrize("extra", [[], ["--emulate-world", "8:1"]])
def test_kshard_process_exits_cleanly_without_close(extra):
    """a world-1 RCCL K-shard run (tools/kshard_native_step.py) that leaves its K-shard, table sets and
    communicator open at exit must end with status 0 -- teardown happens in _lib's atexit hook, while HIP and RCCL
    are still up, not in the runtimes' exit-time destructors."""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "QCE_KSHARD_EMULATE_WORLD", "QCE_NO_EXIT_CLOSE"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "kshard_native_step.py"), "--K", "16", "--B",
                        "8192", "--steps", "3", "--no-close"] + extra, env=env, capture_output=True, text=True,
                       timeout=180)
    assert p.returncode == 0, (p.returncode, p.stderr[-3000:])
    rec = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["vs_single_gpu_rel_fro"] < 1e-12
    assert rec["parity_rel_fro"] < 1e-9


def test_zero_mean_prepare_after_pilot_growth():
    """a zero-mean model prepared with a 16-row pilot matrix, then the 64-row identity (q0 / b grow): the
    grown q0 / b must be zero again whatever address hipMalloc returns -- results vs the oracle at both sizes."""
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import _lib, inputs
    K, N, B = 8, 64, 512
    means, covs, w = inputs.synthetic_model(K, N, seed=9)
    rng = np.random.default_rng(10)
    hp, _ = inputs.scm_generate(B, 1, N, rng, n_path=3)
    h = hp[:, 0, :].astype(complex)
    A = np.eye(N)[::4].astype(complex)  # 16 pilots
    dm = _lib.DeviceModel(None, covs, w, device=0)
    zero = np.zeros((K, N), complex)
    for Ause in (A, None, A, None):
        Aeff = np.eye(N) if Ause is None else Ause
        y = np.ascontiguousarray(inputs.get_observation_nbit(h, 5.0, Aeff, 1, rng=rng), dtype=np.complex128)
        dm.prepare(Ause, 5.0, 1)
        hg = dm.estimate(y)
        ho = O.estimate(zero, covs, w, y, 5.0, N, Aeff, "all", 1)
        assert rel_fro(hg, ho) < 1e-9
    dm.close()
