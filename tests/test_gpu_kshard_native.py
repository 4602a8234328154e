"""The library's own K-shard step (csrc/qce_kshard.hip, include/qce.h qce_comm_* / qce_kshard_*) on the GPU.

* world 1 over a real RCCL communicator (qce_comm_init -> ncclCommInitRank; every collective of the step runs,
  none is skipped at world 1): 'all' and the selective modes on the reference fixtures, the metric geometry
  against the FP64 oracle, the Cholesky error, the exact recombination of flagged rows;
* world 2 and 3 on the one GPU of the box through a host transport (qce_comm_init_host over gloo: RCCL refuses two
  ranks on one device), which runs the same library code path -- chunk layout, reduce-scatter rows, flag words,
  the per-row-shift recombination, the selective modes' all-gathers -- with the collectives staged on the host.

Reference: SURVEY.md §8(b) B3, §8(e) E2; gmm_cplx_bussgang.py:197-243 (modes), :43-46 (the error text);
Bussgang_GMM.py:29-32, :287 (the parallelism this replaces)."""
import datetime
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import MODES, ROOT, case_args, load_model, rel_fro

pytestmark = pytest.mark.gpu

H_TOL = 1e-5  # north-star bar against the reference fixtures


def _prep_args(n_bits, qtype, quantizer):
    from quantized_channel_estimation_amd import _lib
    qk, thr, lab = _lib.QUANT_UNIFORM, None, None
    if n_bits != 1 and not np.isinf(n_bits):
        if qtype == "lloyd":
            qk, thr, lab = _lib.QUANT_LLOYD, np.asarray(quantizer[0], float), np.asarray(quantizer[1], float)
        elif qtype != "uniform":
            qk = _lib.QUANT_OTHER
    return qk, thr, lab


def _mode(m):
    from quantized_channel_estimation_amd import _lib
    if m == "all":
        return _lib.MODE_ALL, 0.0
    if isinstance(m, int):
        return _lib.MODE_TOPN, float(m)
    return _lib.MODE_CUMP, float(m)


def _full_h(rows, h, B):
    """Scatter a rank's (rows, h) back to B rows (NaN elsewhere)."""
    out = np.full((B, h.shape[1]), np.nan + 0j)
    r = np.arange(B) if rows is None else rows.cpu().numpy()
    out[r] = h.cpu().numpy()
    return out, r


# ------------------------------------------------------------------------------------------ world 1, RCCL
@pytest.fixture(scope="module")
def rccl1():
    from quantized_channel_estimation_amd import _lib
    from quantized_channel_estimation_amd.sharding import make_comm
    if _lib.device_count() == 0:
        pytest.fail("no GPU visible for a gpu-marked test")
    comm = make_comm(0, 1, 0, kind="rccl")
    assert comm.kind == _lib.COMM_RCCL
    yield comm
    comm.close()


@pytest.mark.parametrize("mname", ["full", "fullmean", "circ", "bcirc", "synth64"])
def test_world1_rccl_matches_reference_and_single_gpu(rccl1, mname):
    """Every fixture case and mode through qce_kshard_estimate on a world-1 RCCL communicator: within the
    north-star bar of the reference's own h, and equal to the single-GPU library path (1e-11; the selective modes
    take the same lp / selection / filter kernels, argmax to the last bit)."""
    import torch
    from quantized_channel_estimation_amd import _lib
    from quantized_channel_estimation_amd.sharding import ComponentShardEstimator
    fx = load_model(mname)
    est = ComponentShardEstimator(fx["means_cplx"], fx["covs_cplx"], fx["weights"], 0, 1, device=0, comm=rccl1)
    single = _lib.DeviceModel(fx["means_cplx"], fx["covs_cplx"], fx["weights"], device=0)
    torch.cuda.set_device(0)
    for tag in fx["cases"]:
        tag = str(tag)
        y, snr, N, A, n_bits, qtype, quantizer = case_args(fx, tag)
        Ause = None if np.array_equal(A, np.eye(A.shape[0])) else A
        qk, thr, lab = _prep_args(n_bits, qtype, quantizer)
        est.prepare(Ause, snr, n_bits, qk, thr, lab)
        single.prepare(Ause, snr, n_bits, qk, thr, lab)
        yd = torch.from_numpy(np.ascontiguousarray(y)).cuda()
        for mtag, m in MODES.items():
            mode, param = _mode(m)
            for chunks, scatter in ((2, True), (3, False)):
                rows, h = est.estimate(yd, chunks=chunks, scatter=scatter, mode=mode, param=param)
                hg, r = _full_h(rows, h, y.shape[0])
                assert sorted(r.tolist()) == list(range(y.shape[0]))
                err = rel_fro(hg, fx[f"{tag}__hest_{mtag}"])
                assert err < H_TOL, (mname, tag, mtag, err)
                hs = single.estimate(np.ascontiguousarray(y), mode, param)
                e1 = rel_fro(hg, hs)
                assert e1 < (1e-14 if mtag == "top1" else 1e-11), (mname, tag, mtag, chunks, scatter, e1)


def test_world1_rccl_metric_geometry_vs_oracle(rccl1):
    """The metric configuration's geometry (K=128, N=M=64, 1 bit, 5 dB) on a 20k-row batch: FP64 oracle parity on
    512 rows at 1e-9, the single-GPU fused kernel on every row at 1e-12, one timed partial launch per chunk."""
    import torch
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import _lib, inputs
    from quantized_channel_estimation_amd.sharding import ComponentShardEstimator
    K, N, B = 128, 64, 20000
    means, covs, w = inputs.synthetic_model(K, N)
    rng = np.random.default_rng(77)
    hp, _ = inputs.scm_generate(1024, 1, N, rng, n_path=3)
    h = hp[:, 0, :].astype(complex)[rng.integers(0, 1024, size=B)]
    y = np.ascontiguousarray(inputs.get_observation_nbit(h, 5.0, None, 1, rng=rng), dtype=np.complex128)
    est = ComponentShardEstimator(means, covs, w, 0, 1, device=0, comm=rccl1)
    est.prepare(None, 5.0, 1)
    yd = torch.from_numpy(y).cuda()
    est.native.timing(True)
    rows, hk = est.estimate(yd, chunks=2, scatter=True)
    ms, launches = est.native.kernel_ms()
    est.native.timing(False)
    assert launches == 2 and ms > 0.0
    hg, _ = _full_h(rows, hk, B)
    ho = O.estimate(means, covs, w, y[:512], 5.0, N, None, "all", 1)
    assert rel_fro(hg[:512], ho) < 1e-9
    single = _lib.DeviceModel(means, covs, w, device=0)
    single.prepare(None, 5.0, 1)
    assert rel_fro(hg, single.estimate(y)) < 1e-12
    # the argmax mode at this geometry: labels from the gathered (max lp, index) pairs, h bit-identical
    rows, hk = est.estimate(yd, mode=_lib.MODE_TOPN, param=1.0)
    hg1, _ = _full_h(rows, hk, B)
    assert rel_fro(hg1, single.estimate(y, _lib.MODE_TOPN, 1.0)) < 1e-14


@pytest.mark.parametrize("sync", [True, False])
def test_world1_rccl_nonpd_raises_reference_error(rccl1, sync):
    import torch
    from quantized_channel_estimation_amd.sharding import ComponentShardEstimator
    qx = np.load(os.path.join(ROOT, "tests", "golden", "quirks.npz"))
    for tag, nb in (("nonpd_inf", np.inf), ("nonpd_b1", 1)):
        est = ComponentShardEstimator(qx["means_cplx"], qx["bad_covs"], qx["weights"], 0, 1, device=0, comm=rccl1)
        y = torch.from_numpy(np.ascontiguousarray(qx[tag + "__y"])).cuda()
        with pytest.raises(ValueError) as ei:
            est.prepare(None, 20.0, nb)
            est.estimate(y, chunks=2, scatter=True, sync=sync)
            if not sync:
                est.finish()
        assert str(ei.value) == str(qx[tag + "__result"])


def test_world1_rccl_flagged_rows_recombined(rccl1, monkeypatch):
    """Raise the agreed shift (test hook QCE_KSHARD_SHIFT_BIAS) so about half of the rows leave the normal FP64
    range: finish() recombines them exactly (per-row MAX of the running maxima, then the SUM)."""
    import torch
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd.sharding import ComponentShardEstimator
    fx = load_model("fullmean")
    y, snr, N, A, n_bits, qtype, quantizer = case_args(fx, "b1_5")
    href, t = O.estimate(fx["means_cplx"], fx["covs_cplx"], fx["weights"], y, snr, N, A, "all", n_bits, qtype,
                         quantizer, return_tables=True)
    lp = O.weighted_log_prob(y, t["means_y"], t["P"], fx["weights"])
    c = 2 * np.real(O.log_det_cholesky(t["P"])) + np.log(fx["weights"]) - A.shape[0] * np.log(np.pi)
    bias = float(np.median(lp.max(axis=1))) + 667.7 - float(c.max())
    monkeypatch.setenv("QCE_KSHARD_SHIFT_BIAS", repr(bias))
    est = ComponentShardEstimator(fx["means_cplx"], fx["covs_cplx"], fx["weights"], 0, 1, device=0, comm=rccl1)
    est.prepare(None, snr, n_bits)
    yd = torch.from_numpy(np.ascontiguousarray(y)).cuda()
    rows, h = est.estimate(yd, chunks=3, scatter=True)
    hg, _ = _full_h(rows, h, y.shape[0])
    assert rel_fro(hg, href) < 1e-9
    # two superseded flagged steps: the first cannot be repaired any more -> RuntimeError at finish
    est.estimate(yd, chunks=3, scatter=True, sync=False)
    est.estimate(yd, chunks=3, scatter=True, sync=False)
    with pytest.raises(RuntimeError, match="earlier K-shard estimate"):
        est.finish()


# ------------------------------------------------------------------------------------------ world 2/3, host transport
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(target, world, args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + tuple(args) + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=150) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return res


def _host_worker(rank, world, port, mname, q):
    import sys
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import _lib
    from quantized_channel_estimation_amd.sharding import ComponentShardEstimator, make_comm
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=90))
    torch.cuda.set_device(0)
    fx = load_model(mname)
    comm = make_comm(rank, world, 0, kind="host")
    est = ComponentShardEstimator(fx["means_cplx"], fx["covs_cplx"], fx["weights"], rank, world, device=0, comm=comm)
    out = []
    for tag in [str(t) for t in fx["cases"]][:4]:
        y, snr, N, A, n_bits, qtype, quantizer = case_args(fx, tag)
        Ause = None if np.array_equal(A, np.eye(A.shape[0])) else A
        est.prepare(Ause, snr, n_bits, *_prep_args(n_bits, qtype, quantizer))
        yd = torch.from_numpy(np.ascontiguousarray(y)).cuda()
        for mtag, m in MODES.items():
            mode, param = _mode(m)
            for chunks, scatter in ((3, True), (2, False)):
                rows, h = est.estimate(yd, chunks=chunks, scatter=scatter, mode=mode, param=param)
                r = np.arange(y.shape[0]) if rows is None else rows.cpu().numpy()
                ho = O.estimate(fx["means_cplx"], fx["covs_cplx"], fx["weights"], y[r], snr, N, A,
                                m if m == "all" else m, n_bits, qtype, quantizer)
                ref = fx[f"{tag}__hest_{mtag}"][r]
                out.append((tag, mtag, chunks, scatter, r.tolist(), rel_fro(h.cpu().numpy(), ho),
                            rel_fro(h.cpu().numpy(), ref)))
    # exact recombination across ranks: about half of the rows flagged
    y, snr, N, A, n_bits, qtype, quantizer = case_args(fx, str(fx["cases"][0]))
    href, t = O.estimate(fx["means_cplx"], fx["covs_cplx"], fx["weights"], y, snr, N, A, "all", n_bits, qtype,
                         quantizer, return_tables=True)
    lp = O.weighted_log_prob(y, t["means_y"], t["P"], fx["weights"])
    c = 2 * np.real(O.log_det_cholesky(t["P"])) + np.log(fx["weights"]) - A.shape[0] * np.log(np.pi)
    os.environ["QCE_KSHARD_SHIFT_BIAS"] = repr(float(np.median(lp.max(axis=1))) + 667.7 - float(c.max()))
    Ause = None if np.array_equal(A, np.eye(A.shape[0])) else A
    est.prepare(Ause, snr, n_bits, *_prep_args(n_bits, qtype, quantizer))
    del os.environ["QCE_KSHARD_SHIFT_BIAS"]
    rows, h = est.estimate(torch.from_numpy(np.ascontiguousarray(y)).cuda(), chunks=3, scatter=True)
    r = rows.cpu().numpy()
    rep = rel_fro(h.cpu().numpy(), href[r])
    dist.destroy_process_group()
    q.put((rank, out, rep))


@pytest.mark.parametrize("world,mname", [(2, "fullmean"), (3, "full"), (2, "circ")])
def test_host_transport_multirank_all_and_selective_modes(world, mname):
    """2 / 3 ranks on the one GPU, collectives through gloo staged by the library: 'all' (reduce-scatter and
    all-reduce layouts, 3 / 2 chunks) and the selective modes against the FP64 oracle (1e-9; labels and the
    top-n / cumulative-p selections identical) and the reference's own h; flagged rows recombined exactly."""
    res = _run(_host_worker, world, (mname,))
    for m in ("all", "top1", "top3", "p09"):
        for sc in (True, False):
            cover = []
            for rank, out, _ in res:
                for tag, mtag, chunks, scatter, r, eo, er in out:
                    if mtag == m and scatter == sc and tag == out[0][0]:
                        cover += r
            if sc:
                assert sorted(cover) == list(range(len(set(cover)))), (m, sc)
    for rank, out, rep in res:
        for tag, mtag, chunks, scatter, r, eo, er in out:
            # the documented sensitivities (tests/test_gpu_parity.py): 1 bit with a general A (arcsine
            # law near |rho| = 1), and 1 bit on the Fourier path (the dense reference's circulant Cy differs in its
            # last bits along a diagonal) -- 1e-6 / 1e-7; everything else 1e-9
            tol = 1e-6 if tag.startswith("p2_b1") else (1e-7 if mname in ("circ", "bcirc") and tag.startswith("b1") else 1e-9)
            assert eo < tol, (rank, tag, mtag, chunks, scatter, eo)
            assert er < H_TOL, (rank, tag, mtag, chunks, scatter, er)
        tol = 1e-7 if mname in ("circ", "bcirc") else 1e-9  # the first case is 1 bit (see above)
        assert rep < tol, (rank, rep)


def _chol_worker(rank, world, port, sync, q):
    import sys
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from quantized_channel_estimation_amd.sharding import ComponentShardEstimator, make_comm
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=90))
    torch.cuda.set_device(0)
    comm = make_comm(rank, world, 0, kind="host")
    qx = np.load(os.path.join(ROOT, "tests", "golden", "quirks.npz"))
    out = []
    for tag, nb in (("nonpd_inf", np.inf), ("nonpd_b1", 1)):
        est = ComponentShardEstimator(qx["means_cplx"], qx["bad_covs"], qx["weights"], rank, world, device=0,
                                      comm=comm)
        y = torch.from_numpy(np.ascontiguousarray(qx[tag + "__y"])).cuda()
        msg = None
        try:
            est.prepare(None, 20.0, nb)
            est.estimate(y, chunks=2, scatter=True, sync=sync)
            if not sync:
                est.finish()
        except ValueError as e:
            msg = str(e)
        out.append((tag, msg, str(qx[tag + "__result"])))
        dist.barrier()
    dist.destroy_process_group()
    q.put((rank, out))


@pytest.mark.parametrize("sync", [True, False])
def test_host_transport_nonpd_raises_on_every_rank(sync):
    for rank, out in _run(_chol_worker, 2, (sync,)):
        for tag, msg, want in out:
            assert msg == want, (rank, tag, msg)


def test_world1_rccl_double_buffered_snr_sweep(rccl1):
    """Double-buffered tables (qce_kshard_set_spare): an SNR sweep of sync=False steps, each prepare filling the
    table set the previous step did not read while that step runs; every step's h equals the single-GPU library
    result at its own SNR (the reference's script loop, Bussgang_GMM.py:284-287, one estimate per SNR point)."""
    import torch
    from quantized_channel_estimation_amd import _lib
    from quantized_channel_estimation_amd.sharding import ComponentShardEstimator
    fx = load_model("fullmean")
    y, _, N, A, n_bits, qtype, quantizer = case_args(fx, "b1_5")
    yd = torch.from_numpy(np.ascontiguousarray(y)).cuda()
    est = ComponentShardEstimator(fx["means_cplx"], fx["covs_cplx"], fx["weights"], 0, 1, device=0, comm=rccl1,
                                  double_buffer=True)
    single = _lib.DeviceModel(fx["means_cplx"], fx["covs_cplx"], fx["weights"], device=0)
    snrs = [-10.0, 0.0, 5.0, 10.0, 20.0, -5.0]
    outs = []
    for snr in snrs:
        est.prepare(None, snr, 1)
        rows, h = est.estimate(yd, chunks=2, scatter=True, sync=False)
        outs.append(h)  # each step writes its own output tensor
    est.finish()
    torch.cuda.synchronize()
    for snr, h in zip(snrs, outs):
        single.prepare(None, snr, 1)
        assert rel_fro(h.cpu().numpy(), single.estimate(np.ascontiguousarray(y))) < 1e-12, snr


def test_world1_rccl_premul_scales_rows(rccl1, monkeypatch):
    """The SUMs take each shard's rows times e^{M_r - M*} (RCCL PreMulSum, scalar in device memory).  At world 1 the
    factor is 1, so the test hook QCE_KSHARD_GLOBAL_BIAS raises the agreed M* by 2000 nats: the PreMulSum must then
    zero every row (all of them flagged, flags()[0] == B) and finish() recombines them exactly."""
    import torch
    from quantized_channel_estimation_amd import _lib
    from quantized_channel_estimation_amd.sharding import ComponentShardEstimator
    fx = load_model("full")
    y, snr, N, A, n_bits, qtype, quantizer = case_args(fx, str(fx["cases"][0]))
    Ause = None if np.array_equal(A, np.eye(A.shape[0])) else A
    qk, thr, lab = _prep_args(n_bits, qtype, quantizer)
    est = ComponentShardEstimator(fx["means_cplx"], fx["covs_cplx"], fx["weights"], 0, 1, device=0, comm=rccl1)
    single = _lib.DeviceModel(fx["means_cplx"], fx["covs_cplx"], fx["weights"], device=0)
    est.prepare(Ause, snr, n_bits, qk, thr, lab)
    single.prepare(Ause, snr, n_bits, qk, thr, lab)
    yd = torch.from_numpy(np.ascontiguousarray(y)).cuda()
    rows, h = est.estimate(yd, chunks=2, scatter=True)
    assert est.native.flags()[0] == 0.0
    monkeypatch.setenv("QCE_KSHARD_GLOBAL_BIAS", "2000")
    rows, h = est.estimate(yd, chunks=2, scatter=True)
    assert est.native.flags()[0] == y.shape[0]
    hg, _ = _full_h(rows, h, y.shape[0])
    assert rel_fro(hg, single.estimate(np.ascontiguousarray(y))) < 1e-12


def test_world1_rccl_lagging_comm_stream(rccl1, monkeypatch):
    """the send rows alternate between two buffers, so step t+2 refills the buffer step t's collectives
    read.  Hold the communication stream 3 ms per step (QCE_KSHARD_CS_DELAY_US) so the collectives lag far behind the
    compute stream over three sync=False steps at different SNRs, with double-buffered tables: every step's h must
    still equal the single-GPU result at its SNR (step t+2 waits for step t's communication-stream work)."""
    import torch
    from quantized_channel_estimation_amd import _lib
    from quantized_channel_estimation_amd.sharding import ComponentShardEstimator
    fx = load_model("fullmean")
    y, _, N, A, n_bits, qtype, quantizer = case_args(fx, "b1_5")
    yd = torch.from_numpy(np.ascontiguousarray(y)).cuda()
    est = ComponentShardEstimator(fx["means_cplx"], fx["covs_cplx"], fx["weights"], 0, 1, device=0, comm=rccl1,
                                  double_buffer=True)
    single = _lib.DeviceModel(fx["means_cplx"], fx["covs_cplx"], fx["weights"], device=0)
    monkeypatch.setenv("QCE_KSHARD_CS_DELAY_US", "3000")
    snrs = [-10.0, 20.0, 0.0, 10.0]
    outs = []
    for snr in snrs:
        est.prepare(None, snr, 1)
        rows, h = est.estimate(yd, chunks=2, scatter=False, sync=False)
        outs.append(h)
    est.finish()
    torch.cuda.synchronize()
    for snr, h in zip(snrs, outs):
        single.prepare(None, snr, 1)
        assert rel_fro(h.cpu().numpy(), single.estimate(np.ascontiguousarray(y))) < 1e-12, snr


def _interleave_worker(rank, world, port, q):
    """Two ranks, host transport, double-buffered tables: prepare(t+1) issued between the sync=False estimates t and
    t+1 on both ranks, one finish at the end."""
    import sys
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    from quantized_channel_estimation_amd import _lib
    from quantized_channel_estimation_amd.sharding import ComponentShardEstimator, make_comm
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=90))
    torch.cuda.set_device(0)
    fx = load_model("fullmean")
    y, _, N, A, n_bits, qtype, quantizer = case_args(fx, "b1_5")
    yd = torch.from_numpy(np.ascontiguousarray(y)).cuda()
    comm = make_comm(rank, world, 0, kind="host")
    est = ComponentShardEstimator(fx["means_cplx"], fx["covs_cplx"], fx["weights"], rank, world, device=0, comm=comm,
                                  double_buffer=True)
    single = _lib.DeviceModel(fx["means_cplx"], fx["covs_cplx"], fx["weights"], device=0)
    snrs = [-10.0, 5.0, 20.0]
    outs = []
    est.prepare(None, snrs[0], 1)
    for i, snr in enumerate(snrs):
        rows, h = est.estimate(yd, chunks=2, scatter=True, sync=False)
        outs.append((rows, h))
        if i + 1 < len(snrs):
            est.prepare(None, snrs[i + 1], 1)  # the next SNR's tables while this step is in flight
    est.finish()
    torch.cuda.synchronize()
    errs = []
    for snr, (rows, h) in zip(snrs, outs):
        single.prepare(None, snr, 1)
        r = rows.cpu().numpy()
        errs.append(rel_fro(h.cpu().numpy(), single.estimate(np.ascontiguousarray(y))[r]))
    est.native.close()
    comm.close()
    dist.destroy_process_group()
    q.put((rank, errs))


def test_host_transport_prepare_interleaved_between_async_steps():
    """a prepare between two sync=False estimates on both ranks (double-buffered tables), 2 ranks."""
    res = _run(_interleave_worker, 2, ())
    assert sorted(r for r, _ in res) == [0, 1]
    for rank, errs in res:
        assert max(errs) < 1e-12, (rank, errs)


def test_bench_native_two_ranks_on_one_gpu():
    """the driver's multi-GPU command (bench.py --gpus 2, native backend) end to end on the one-GPU
    box: launch_ranks, gloo rendezvous, the library's communicator (host transport: the ranks share the GPU),
    qce_kshard_prepare / estimate / finish with double-buffered tables, MAX-over-ranks timing, teardown.  Metric
    geometry (K=128, N=M=64) on a 20k batch."""
    import json
    import subprocess
    import sys
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup",
                        "2", "--batch", "20000", "--cpu-seconds", "0", "--no-extras"], env=env, capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    r = json.loads(lines[0])
    assert r["world_size"] == 2 and r["n_gpus"] == 2
    assert "libqce" in r["config"]["collectives"] and r["config"]["parallelism"] == "kshard2"
    assert r["parity"]["rel_fro"] < 1e-9
    assert r["value"] > 0
