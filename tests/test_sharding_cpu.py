"""Multi-process (gloo, world_size 2 and 3) checks of the component-shard combine on CPU.

The per-shard partials (running max m, s = sum e^{lp-m}, acc = sum e^{lp-m} h_k) are produced by
the FP64 oracle here (the GPU produces them with qce_estimate_partial); the distributed combine
(one SUM all-reduce + the underflow fallback) must reproduce the full 'all'-mode estimate."""
import datetime
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT, load_model, case_args, rel_fro


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _partials(fx, tag, lo, hi, lp_shift=0.0):
    from oracle import qce_oracle as O
    y, snr, N, A, n_bits, qtype, quantizer = case_args(fx, tag)
    h, t = O.estimate(fx["means_cplx"], fx["covs_cplx"], fx["weights"], y, snr, N, A, "all", n_bits, qtype,
                      quantizer, return_tables=True)
    lp = O.weighted_log_prob(y, t["means_y"], t["P"], fx["weights"]) - lp_shift
    c = 2 * np.real(O.log_det_cholesky(t["P"])) + np.log(fx["weights"]) - A.shape[0] * np.log(np.pi) - lp_shift
    hk = np.einsum("knm,bm->bkn", t["W"], y) + t["b"][None]
    sl = slice(lo, hi)
    m = lp[:, sl].max(axis=1)
    e = np.exp(lp[:, sl] - m[:, None])
    s = e.sum(axis=1)
    acc = np.einsum("bk,bkn->bn", e, hk[:, sl])
    acc_f = np.empty((acc.shape[0], 2 * N), np.float32)
    acc_f[:, 0::2], acc_f[:, 1::2] = acc.real, acc.imag
    return m, s, acc_f, float(c.max()), h


def _worker(rank, world, port, tag, shift, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    sys.path.insert(0, ROOT)
    from quantized_channel_estimation_amd.sharding import combine_partials_dist, component_slices
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    fx = load_model("fullmean")
    K, N = int(fx["K"]), int(fx["N"])
    lo, hi = component_slices(K, world)[rank]
    m, s, acc, cmax, h_ref = _partials(fx, tag, lo, hi)
    hc = combine_partials_dist(torch.from_numpy(m), torch.from_numpy(s), torch.from_numpy(acc), cmax + shift, N)
    err = rel_fro(hc.numpy(), h_ref)
    dist.destroy_process_group()
    q.put((rank, err))


@pytest.mark.parametrize("world,tag,shift", [(2, "b1_5", 0.0), (3, "u2_m10", 0.0), (2, "l3_20", 0.0),
                                             (2, "b1_5", 900.0)])
def test_component_shard_combine_gloo(world, tag, shift):
    """shift = 900 raises the shift M* so every e^{m - M*} underflows: the single all-reduce then sums
    zeros and the MAX-then-SUM fallback must take over."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, tag, shift, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, err in res:
        # partial accumulators are FP32 (as the kernel writes them)
        assert err < 1e-6, (rank, err)


def test_slices_cover_and_balance():
    from quantized_channel_estimation_amd.sharding import component_slices, combine_partials_numpy
    for K in (1, 7, 128, 256):
        for W in (1, 2, 3, 8):
            sl = component_slices(K, W)
            assert sl[0][0] == 0 and sl[-1][1] == K
            assert all(a[1] == b[0] for a, b in zip(sl, sl[1:]))
            sizes = [b - a for a, b in sl]
            assert max(sizes) - min(sizes) <= 1
    fx = load_model("full")
    parts = []
    for lo, hi in [(0, 5), (5, 16)]:
        m, s, acc, _, h_ref = _partials(fx, "b1_5", lo, hi)
        parts.append((m, s, acc))
    assert rel_fro(combine_partials_numpy(parts, int(fx["N"])), h_ref) < 1e-6


# ---- pipelined K-shard estimator (chunked, shifted packed partials, async reduce-scatter / all-reduce) ----
class _OracleShard:
    """Stand-in for one rank's DeviceModel: the FP64 oracle's partial of components [lo, hi) in the
    formats qce_estimate_partial_shifted / qce_estimate_partial_f64 / qce_cconst_max return (torch CPU tensors)."""
    device_type = "cpu"

    def __init__(self, fx, tag, lo, hi, chol_fail=False, raise_at=None):
        from oracle import qce_oracle as O
        y, snr, N, A, n_bits, qtype, quantizer = case_args(fx, tag)
        h, t = O.estimate(fx["means_cplx"], fx["covs_cplx"], fx["weights"], y, snr, N, A, "all", n_bits, qtype,
                          quantizer, return_tables=True)
        self.lp_all = O.weighted_log_prob(y, t["means_y"], t["P"], fx["weights"])
        self.lp = self.lp_all[:, lo:hi]
        self.hk = (np.einsum("knm,bm->bkn", t["W"], y) + t["b"][None])[:, lo:hi]
        c = 2 * np.real(O.log_det_cholesky(t["P"])) + np.log(fx["weights"]) - A.shape[0] * np.log(np.pi)
        self.c = c[lo:hi]
        self.N, self.y, self.h = N, y, h
        self.chol_fail = chol_fail
        # where the library surfaces a failed factorisation as ValueError instead (its deferred status read by a
        # later call): None (only the +inf shift), "cconst" or "partial"
        self.raise_at = raise_at if chol_fail else None
        self._row = {self.y[i].tobytes(): i for i in range(self.y.shape[0])}

    def cconst(self):
        return self.c

    def prepare(self, *a, **kw):
        pass

    def cconst_max(self, out=None, stream=None):
        # the kernel writes +inf when a Cholesky factorisation of this shard failed (k_cconst_max)
        if self.raise_at == "cconst":
            from quantized_channel_estimation_amd import _lib
            raise ValueError(_lib.CHOL_MESSAGE)
        out.fill_(float("inf") if self.chol_fail else float(np.max(self.c)))
        return out

    def _rows(self, y):
        import torch
        yn = y.numpy() if isinstance(y, torch.Tensor) else y
        return np.array([self._row[r.tobytes()] for r in yn], dtype=np.int64)

    def partial64(self, y, stream=None):
        import torch
        sl = self._rows(y)
        lp = self.lp[sl]
        m = lp.max(axis=1)
        e = np.exp(lp - m[:, None])
        acc = np.einsum("bk,bkn->bn", e, self.hk[sl])
        a = np.empty((acc.shape[0], 2 * self.N))
        a[:, 0::2], a[:, 1::2] = acc.real, acc.imag
        return torch.from_numpy(m), torch.from_numpy(e.sum(axis=1)), torch.from_numpy(a)

    def partial_shifted(self, y, shift, out=None, stream=None):
        import torch
        if self.raise_at == "partial":
            from quantized_channel_estimation_amd import _lib
            raise ValueError(_lib.CHOL_MESSAGE)
        m, s, a = (t.numpy() for t in self.partial64(y))
        sh = float(shift[0]) if isinstance(shift, torch.Tensor) else float(shift)  # (mock only: no kernel here)
        with np.errstate(under="ignore", over="ignore"):
            sc = np.exp(m - sh)
        buf = np.concatenate([(s * sc)[:, None], np.zeros((m.shape[0], 1)), a * sc[:, None]], axis=1)
        out.copy_(torch.from_numpy(buf))
        return out


def _make_est(rank, world, fx, tag, chol_fail=False, raise_at=None):
    from quantized_channel_estimation_amd.sharding import ComponentShardEstimator, component_slices
    K = int(fx["K"])
    lo, hi = component_slices(K, world)[rank]
    est = ComponentShardEstimator.__new__(ComponentShardEstimator)
    est.rank, est.world, est.lo, est.hi, est.group, est._bufs = rank, world, lo, hi, None, {}
    est._pending = est._flag_acc = None
    est._chol_local = False
    est.shift = None
    est.dev = _OracleShard(fx, tag, lo, hi, chol_fail=chol_fail, raise_at=raise_at)
    est.N = est.dev.N
    return est


def _pipe_worker(rank, world, port, tag, shift, chunks, scatter, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    sys.path.insert(0, ROOT)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    fx = load_model("fullmean")
    est = _make_est(rank, world, fx, tag)
    est.prepare(None, 0.0, 1)  # shift = MAX over ranks of max c_k, on the "device" (a CPU tensor here)
    if shift == "half":
        # raise the shift so the rows with the smaller max lp leave the normal range (a subset is flagged)
        mb = est.dev.lp_all.max(axis=1)
        est.shift += float(np.median(mb) - est.shift.item()) + 667.7
    else:
        est.shift += shift
    y = torch.from_numpy(est.dev.y)
    rows, h = est.estimate(y, chunks=chunks, scatter=scatter)
    ref = est.dev.h if rows is None else est.dev.h[rows.numpy()]
    err = rel_fro(h.numpy(), ref)
    n = h.shape[0]
    # every row is owned by exactly one rank under scatter
    cnt = torch.tensor([n], dtype=torch.float64)
    dist.all_reduce(cnt)
    dist.destroy_process_group()
    q.put((rank, err, int(cnt.item()), y.shape[0]))


@pytest.mark.parametrize("world,tag,shift,chunks,scatter", [
    (2, "b1_5", 0.0, 3, True), (3, "u2_m10", 0.0, 4, True), (2, "l3_20", 0.0, 1, False),
    (2, "b1_5", 900.0, 2, True), (3, "b1_5", 900.0, 2, False), (2, "b1_5", "half", 3, True),
    (3, "u2_m10", "half", None, True), (2, "l3_20", "half", 2, False)])
def test_pipelined_component_shard_gloo(world, tag, shift, chunks, scatter):
    """The pipelined K-shard estimator over gloo: chunked shifted partials, one SUM collective per chunk
    (reduce-scatter or all-reduce), FP64 throughout; shift + 900 flags every row, "half" about half of them
    (each rank flags only rows it owns under reduce-scatter): only the flagged rows are recombined exactly."""
    _run(_pipe_worker, world, (tag, shift, chunks, scatter))


def _run(target, world, args, check=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + tuple(args) + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    if check is not None:
        return check(res)
    scatter = args[-1]
    for rank, err, total, B in res:
        assert err < 1e-12, (rank, err)
        assert total == (B if scatter else B * world)


def _nosync_worker(rank, world, port, steps, q):
    """sync=False steps make no host read of a device value; finish() makes one (the flag word)."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    sys.path.insert(0, ROOT)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    fx = load_model("fullmean")
    est = _make_est(rank, world, fx, "b1_5")
    y = torch.from_numpy(est.dev.y)
    est.prepare(None, 0.0, 1)
    counts = {"n": 0}
    names = ("item", "tolist", "cpu", "numpy", "__float__", "__int__", "__bool__", "__index__")
    saved = {n: getattr(torch.Tensor, n) for n in names}

    def counting(fn):
        def f(*a, **kw):
            counts["n"] += 1
            return fn(*a, **kw)
        return f
    part = est.dev.partial_shifted
    orig_partial = est.dev.partial_shifted

    def quiet_partial(yy, shift, out=None, stream=None):  # the mock's own host reads are not the estimator's
        for n in names:
            setattr(torch.Tensor, n, saved[n])
        try:
            return orig_partial(yy, shift, out=out, stream=stream)
        finally:
            for n in names:
                setattr(torch.Tensor, n, counting(saved[n]))
    est.dev.partial_shifted = quiet_partial
    for n in names:
        setattr(torch.Tensor, n, counting(saved[n]))
    try:
        for _ in range(steps):
            est.estimate(y, chunks=2, scatter=True, sync=False)
        per_steps = counts["n"]
        counts["n"] = 0
        rows, h = est.finish()
        at_finish = counts["n"]
    finally:
        for n in names:
            setattr(torch.Tensor, n, saved[n])
    est.dev.partial_shifted = part
    err = rel_fro(h.numpy(), est.dev.h[rows.numpy()])
    dist.destroy_process_group()
    q.put((rank, per_steps, at_finish, err))


def test_kshard_no_host_sync_per_step_gloo():
    def check(res):
        for rank, per_steps, at_finish, err in res:
            assert per_steps == 0, (rank, per_steps)
            assert at_finish <= 2, (rank, at_finish)  # flags of the last step + of the whole run
            assert err < 1e-12
    _run(_nosync_worker, 2, (3,), check)


def _chol_worker(rank, world, port, sync, raise_at, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    sys.path.insert(0, ROOT)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    fx = load_model("fullmean")
    est = _make_est(rank, world, fx, "b1_5", chol_fail=(rank == world - 1), raise_at=raise_at)
    est.prepare(None, 0.0, 1)
    y = torch.from_numpy(est.dev.y)
    msg = None
    try:
        est.estimate(y, chunks=2, scatter=True, sync=sync)
        if not sync:
            est.finish()
    except ValueError as e:
        msg = str(e)
    dist.destroy_process_group()
    q.put((rank, msg))


@pytest.mark.parametrize("sync,raise_at", [(True, None), (False, None), (True, "partial"), (False, "cconst")])
def test_kshard_cholesky_failure_raises_on_every_rank_gloo(sync, raise_at):
    """A non-PD Cr_k on one rank (its shard shift is +inf) reaches every rank through the shift's MAX and the
    step's flag word: each raises the reference's ValueError text (gmm_cplx_bussgang.py:43-46; quirks.npz).
    raise_at: the library reported the failure from a later device call on that rank instead -- the rank must
    still join every collective of the step (no hang) and all ranks raise together."""
    q = np.load(os.path.join(ROOT, "tests", "golden", "quirks.npz"))
    want = str(q["nonpd_b1__result"])

    def check(res):
        for rank, msg in res:
            assert msg == want, (rank, msg)
    _run(_chol_worker, 3, (sync, raise_at), check)


def test_chunk_bounds_cover():
    from quantized_channel_estimation_amd.sharding import chunk_bounds
    for B in (1, 7, 100, 1001):
        for world in (1, 2, 3, 8):
            for ch in (1, 3, 4):
                for sc in (True, False):
                    b = chunk_bounds(B, ch, world, sc)
                    assert b[0][0] == 0 and b[-1][1] == B
                    assert all(x[1] == y[0] for x, y in zip(b, b[1:]))
                    if sc:
                        assert all((hi - lo) % world == 0 for lo, hi in b[:-1])


def test_bench_launcher_gloo_world2():
    """`bench.py --gpus 2` starts its own two ranks (before any GPU call), they rendezvous on 127.0.0.1,
    reduce the per-rank time with MAX and rank 0 prints one JSON line (CPU rehearsal, gloo)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, r.stdout
    d = json.loads(line[0])
    assert d["world_size"] == 2 and d["n_gpus"] == 2 and sorted(d["ranks"]) == [0, 1]
    assert abs(d["max_elapsed"] - 0.02) < 1e-12


def _two_flagged_worker(rank, world, port, q):
    """two sync=False steps that both have flagged rows -- the first one was superseded (its h already
    handed back with NaN rows), so finish() must raise instead of silently repairing only the last step."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    sys.path.insert(0, ROOT)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    fx = load_model("fullmean")
    est = _make_est(rank, world, fx, "b1_5")
    est.prepare(None, 0.0, 1)
    est.shift += 900.0  # every row flagged, in both steps
    y = torch.from_numpy(est.dev.y)
    est.estimate(y, chunks=2, scatter=True, sync=False)
    est.estimate(y, chunks=2, scatter=True, sync=False)
    msg = None
    try:
        est.finish()
    except RuntimeError as e:
        msg = str(e)
    # a single flagged step is still repaired exactly
    est.estimate(y, chunks=2, scatter=True, sync=False)
    rows, h = est.finish()
    err = rel_fro(h.numpy(), est.dev.h[rows.numpy()])
    dist.destroy_process_group()
    q.put((rank, msg, err))


def test_kshard_superseded_flagged_step_raises_gloo():
    def check(res):
        for rank, msg, err in res:
            assert msg is not None and "earlier K-shard estimate" in msg, (rank, msg)
            assert err < 1e-12, (rank, err)
    _run(_two_flagged_worker, 2, (), check)


def test_library_kshard_layout_matches_python():
    """qce_kshard_rows / qce_kshard_slice (host-only entry points of the library's K-shard step) give the same
    component split and per-rank row layout as sharding.component_slices / chunk_bounds."""
    from quantized_channel_estimation_amd import _lib, build
    from quantized_channel_estimation_amd.sharding import chunk_bounds, component_slices
    build.build()
    for K in (2, 7, 128, 256):
        for world in (1, 2, 3, 8):
            if K < world:
                continue
            for r in range(world):
                assert _lib.kshard_slice(K, world, r) == component_slices(K, world)[r]
    for B in (1, 7, 100, 1001, 100000):
        for world in (1, 2, 3, 8):
            for ch in (1, 2, 3, 4):
                for sc in (True, False):
                    b = chunk_bounds(B, ch, world, sc)
                    seen = []
                    for r in range(world):
                        lib = _lib.kshard_rows(B, ch, world, r, sc)
                        assert len(lib) == len(b)
                        for (lo, hi), (a, e) in zip(b, lib):
                            if sc:
                                q = -(-(hi - lo) // world)
                                assert a == lo + r * q and e == min(hi, a + q) or (e == a and a >= hi)
                            else:
                                assert (a, e) == (lo, hi)
                        seen += [i for a, e in lib for i in range(a, e)]
                    if sc:
                        assert sorted(seen) == list(range(B))
