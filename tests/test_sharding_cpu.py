"""Multi-process (gloo, world_size 2 and 3) checks of the component-shard combine on CPU.

The per-shard partials (running max m, s = sum e^{lp-m}, acc = sum e^{lp-m} h_k) are produced by
the FP64 oracle here (the GPU produces them with qce_estimate_partial); the distributed combine
(one SUM all-reduce + the underflow fallback) must reproduce the full 'all'-mode estimate."""
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
    dist.init_process_group("gloo", rank=rank, world_size=world)
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
    formats qce_estimate_partial_shifted / qce_estimate_partial_f64 return (torch CPU tensors)."""

    def __init__(self, fx, tag, lo, hi):
        from oracle import qce_oracle as O
        y, snr, N, A, n_bits, qtype, quantizer = case_args(fx, tag)
        h, t = O.estimate(fx["means_cplx"], fx["covs_cplx"], fx["weights"], y, snr, N, A, "all", n_bits, qtype,
                          quantizer, return_tables=True)
        self.lp = O.weighted_log_prob(y, t["means_y"], t["P"], fx["weights"])[:, lo:hi]
        self.hk = (np.einsum("knm,bm->bkn", t["W"], y) + t["b"][None])[:, lo:hi]
        c = 2 * np.real(O.log_det_cholesky(t["P"])) + np.log(fx["weights"]) - A.shape[0] * np.log(np.pi)
        self.c = c[lo:hi]
        self.N, self.y, self.h = N, y, h

    def cconst(self):
        return self.c

    def _rows(self, y):
        import torch
        # y is a slice of the fixture batch: find its row offset by identity of the data
        yn = y.numpy() if isinstance(y, torch.Tensor) else y
        for off in range(self.y.shape[0] - yn.shape[0] + 1):
            if np.array_equal(self.y[off:off + yn.shape[0]], yn):
                return slice(off, off + yn.shape[0])
        raise AssertionError("unknown rows")

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
        m, s, a = (t.numpy() for t in self.partial64(y))
        sc = np.exp(m - shift)
        buf = np.concatenate([(s * sc)[:, None], np.zeros((m.shape[0], 1)), a * sc[:, None]], axis=1)
        import torch
        out.copy_(torch.from_numpy(buf))
        return out


def _pipe_worker(rank, world, port, tag, shift, chunks, scatter, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    sys.path.insert(0, ROOT)
    from quantized_channel_estimation_amd.sharding import ComponentShardEstimator, component_slices
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fx = load_model("fullmean")
    K = int(fx["K"])
    lo, hi = component_slices(K, world)[rank]
    est = ComponentShardEstimator.__new__(ComponentShardEstimator)
    est.rank, est.world, est.lo, est.hi, est.group, est._bufs = rank, world, lo, hi, None, {}
    est.dev = _OracleShard(fx, tag, lo, hi)
    est.N = est.dev.N
    t = torch.tensor([float(np.max(est.dev.cconst()))], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    est.shift = float(t.item()) + shift
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
    (2, "b1_5", 900.0, 2, True), (3, "b1_5", 900.0, 2, False)])
def test_pipelined_component_shard_gloo(world, tag, shift, chunks, scatter):
    """The pipelined K-shard estimator over gloo: chunked shifted partials, one SUM collective per chunk
    (reduce-scatter or all-reduce), FP64 throughout; shift + 900 forces the underflow fallback."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(r, world, port, tag, shift, chunks, scatter, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, err, total, B in res:
        assert err < 1e-12, (rank, err)
        assert total == (B if scatter else B * world)


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
