"""Multi-GPU decomposition of the estimate path (one process per GPU, torch.distributed over RCCL).

The reference's only parallelism is a process pool over SNR points (Bussgang_GMM.py:29-32, :287);
here one SNR point's batch is split over the GPUs of a node, two ways:

* **component shards** (``ComponentShardEstimator``, the north-star split): rank g holds the
  components K_g.  The shift M* = max_k c_k over ALL components (c_k = log w_k + 2 log det P_k
  - M log pi >= lp_bk because the quad form is >= 0; one scalar MAX all-reduce per SNR) is common
  to every shard, so each rank's partial can be written already scaled,
  row b = [s_b e^{m_b - M*}, 0, acc_b e^{m_b - M*}] (``qce_estimate_partial_shifted``, FP64), and ONE
  SUM collective of these (B, 2N+2) rows gives h_b = acc / s.  The batch is cut into chunks; chunk
  i's collective (reduce-scatter by default: each rank keeps its slice of the rows, half the bytes
  of an all-reduce) is issued asynchronously and runs on RCCL's stream while chunk i+1's partial
  kernel runs on the compute stream.  Rows whose shifted sum leaves the normal FP64 range (max lp more
  than ~667 below M*) are flagged on the device; one tiny MAX all-reduce per step agrees on a flag word
  (flagged rows, Cholesky failure on any rank) that the host reads once at the caller's sync point
  (``finish``), and only the flagged rows are recombined exactly (MAX of m, then SUM).  The collectives
  per step: the per-chunk SUM (reduce-scatter) and the 2-double flag MAX; per SNR point: the shift MAX.
* **batch shards** (``BatchShardEstimator``): every rank holds the whole mixture and estimates a
  disjoint slice of the observations.  No data-path collective — the samples are independent (the
  configuration for the HBM-bound Fourier paths, where a K-shard collective costs more than the
  kernel).
"""
import math

import numpy as np

from . import _lib

# A row whose shifted sum falls below this is recombined exactly: above it every term that matters is a normal
# double (DBL_MIN = 2.2e-308), so the shifted sums carry full FP64 precision.
UNDERFLOW_S = 1e-290


def combine_partials_numpy(parts, N):
    """Host combine of component-shard partials [(m, s, acc), ...] -> h (B, N) complex128."""
    ms = np.stack([np.asarray(p[0]) for p in parts])
    mx = ms.max(axis=0)
    s = np.zeros_like(mx)
    acc = np.zeros((mx.shape[0], 2 * N))
    for (m, sg, ag) in parts:
        sc = np.exp(np.asarray(m) - mx)
        s += np.asarray(sg) * sc
        acc += np.asarray(ag, dtype=np.float64) * sc[:, None]
    acc /= s[:, None]
    return acc[:, 0::2] + 1j * acc[:, 1::2]


def combine_packed_numpy(packed_parts):
    """Host combine of shifted packed partials [(B, 2N+2), ...] (same shift) -> h (B, N)."""
    tot = np.sum([np.asarray(p, dtype=np.float64) for p in packed_parts], axis=0)
    acc = tot[:, 2:] / tot[:, :1]
    return acc[:, 0::2] + 1j * acc[:, 1::2]


def component_slices(K, world):
    """Contiguous, balanced component ranges per rank."""
    base, rem = divmod(K, world)
    out, lo = [], 0
    for r in range(world):
        hi = lo + base + (1 if r < rem else 0)
        out.append((lo, hi))
        lo = hi
    return out


def batch_slices(B, world):
    return component_slices(B, world)


def combine_partials_dist(m, s, acc, shift, N, group=None):
    """Exact distributed combine of one rank's unshifted partial (torch tensors on this rank's device):
    m, s (B,) float64, acc (B, 2N) float32/float64, shift = the global M*.  One SUM all-reduce of the
    rescaled rows; rows that underflow under M* take the MAX-then-SUM path.  h (B, N) complex128 on every
    rank.  (The pipelined path of ComponentShardEstimator uses this only as its underflow fallback.)"""
    import torch
    import torch.distributed as dist
    B = m.shape[0]
    buf = torch.empty((B, 2 * N + 1), dtype=torch.float64, device=m.device)
    sc = torch.exp(m - shift)
    buf[:, 0] = s * sc
    buf[:, 1:] = acc.to(torch.float64) * sc[:, None]
    dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    bad = buf[:, 0] < UNDERFLOW_S
    nbad = bad.sum()
    dist.all_reduce(nbad, op=dist.ReduceOp.MAX, group=group)  # tiny: agree on the fallback
    if int(nbad.item()) > 0:
        idx = torch.nonzero(bad, as_tuple=False).flatten()
        # underflow guard: exact two-step combine for the affected rows (every rank has the same rows)
        mm = m[idx].clone()
        dist.all_reduce(mm, op=dist.ReduceOp.MAX, group=group)
        sc2 = torch.exp(m[idx] - mm)
        sub = torch.empty((idx.numel(), 2 * N + 1), dtype=torch.float64, device=m.device)
        sub[:, 0] = s[idx] * sc2
        sub[:, 1:] = acc[idx].to(torch.float64) * sc2[:, None]
        dist.all_reduce(sub, op=dist.ReduceOp.SUM, group=group)
        buf[idx] = sub
    out = buf[:, 1:] / buf[:, :1]
    return torch.complex(out[:, 0::2].contiguous(), out[:, 1::2].contiguous())


def chunk_bounds(B, chunks, world, scatter):
    """Row ranges of the pipeline chunks; with scatter every chunk but the last has a multiple of
    `world` rows and the last one is padded up to one (reduce_scatter splits rows evenly)."""
    chunks = max(1, min(int(chunks), max(1, B // max(world, 1))))
    step = -(-B // chunks)
    if scatter:
        step = -(-step // world) * world
    out, lo = [], 0
    while lo < B:
        hi = min(B, lo + step)
        out.append((lo, hi))
        lo = hi
    return out


def _packed_to_complex(rows):
    import torch
    acc = rows[:, 2:] / rows[:, :1]
    return torch.complex(acc[:, 0::2].contiguous(), acc[:, 1::2].contiguous())


def default_chunks(world):
    """Pipeline chunks per batch: 1.  Per rank on one MI355X through qce_kshard_* (profiles/r05_kshard_rank16.jsonl,
    r05_kshard_rank_cfg4.jsonl): 1.22 / 1.34 ms per step with 1 / 2 chunks at the metric's K = 16 per rank, 5.36 /
    5.60 ms at cfg4's K = 32 -- a second chunk adds a launch tail and a merge to every step.  With the library's
    send rows alternating between two buffers, step t's reduce-scatter already runs beside step t+1's kernel (on the
    CUs the shard's grid leaves free, QCE_OPT_RESERVE_CUS), so a chunk split buys no overlap in a run of steps."""
    return 1


class ComponentShardEstimator:
    """K-sharded 'all'-mode estimator: this rank's slice of the mixture on its own GPU.

    Per step the host enqueues the chunk kernels and collectives and one tiny MAX all-reduce of a flag word
    [rows whose shifted sum underflowed, Cholesky failure on any rank]; with ``sync=False`` it returns without
    waiting for the device, and ``finish()`` (the caller's natural sync point) reads the flag word once, raises the
    reference's ValueError for a failed factorisation (gmm_cplx_bussgang.py:43-46) and recombines the flagged rows
    exactly.  ``sync=True`` (default) is estimate + finish.

    With ``comm`` (a ``_lib.Comm``, see ``make_comm``) the whole step runs inside the library (qce_kshard_*: the
    collectives are RCCL calls of libqce, or a host transport), including the selective modes; without it the step
    is orchestrated here over torch.distributed (the gloo rehearsal path of the CPU tests)."""

    native = None  # the library's K-shard step (a _lib.KShard) when built with a communicator
    _native_rows = None
    _idx_cache = None  # {(row ranges, device): global row indices} of the last layout

    def __init__(self, means_cplx, covs_cplx, weights, rank, world, device=0, group=None, precision="f64", comm=None,
                 double_buffer=False):
        K = np.asarray(covs_cplx).shape[0]
        self.K = K
        self.rank, self.world = rank, world
        self.lo, self.hi = component_slices(K, world)[rank]
        sl = slice(self.lo, self.hi)
        means = None if means_cplx is None else np.asarray(means_cplx)[sl]
        self.dev = _lib.DeviceModel(means, np.asarray(covs_cplx)[sl], np.asarray(weights)[sl], device=device)
        if precision != "f64":
            self.dev.set_precision(precision)
        self.N = self.dev.N
        self.group = group
        self.shift = None
        self._bufs = {}
        self._pending = None
        self._flag_acc = None
        self._chol_local = False
        if comm is not None:
            if (comm.rank, comm.world) != (rank, world):
                raise ValueError("communicator rank / world differ from the estimator's")
            self.native = _lib.KShard(self.dev, comm, K)
            if double_buffer:  # a second table set: the next prepare overlaps the current step (qce_kshard_set_spare)
                spare = _lib.DeviceModel(means, np.asarray(covs_cplx)[sl], np.asarray(weights)[sl], device=device)
                if precision != "f64":
                    spare.set_precision(precision)
                self.native.set_spare(spare)

    def close(self):
        """Release the library's K-shard step and this rank's table sets (the communicator stays the caller's).  Call
        it before the process ends: teardown left to exit-time destructors is what VERDICT r5 #4 traced a crash to."""
        if self.native is not None:
            spare = getattr(self.native, "spare", None)
            self.native.close()
            if spare is not None:
                spare.close()
        self.dev.close()
        self._bufs = {}

    def _on_gpu(self):
        return getattr(self.dev, "device_type", "cuda") == "cuda"

    def prepare(self, A, snr_db, n_bits, quant_kind=_lib.QUANT_UNIFORM, thresholds=None, labels=None, stream=None):
        """Per-rank prepare of its components and the common shift M* (one scalar MAX all-reduce).  The shift stays
        on the device: this rank's max c_k (+inf if one of its Cholesky factorisations failed) is written by a kernel
        on the prepare's stream, and the all-reduce is ordered behind it -- no host round trip per SNR point."""
        import torch
        import torch.distributed as dist
        if self.native is not None:  # ordered on torch's current stream unless told otherwise (as estimate())
            s = stream if stream is not None else torch.cuda.current_stream(torch.device("cuda", self.dev.device)
                                                                            ).cuda_stream
            self.native.prepare(A, snr_db, n_bits, quant_kind, thresholds, labels, stream=s)
            return
        if self._on_gpu():
            dev = torch.device("cuda", self.dev.device)
            cur = torch.cuda.current_stream(dev)
            s = stream if stream is not None else cur.cuda_stream
        else:
            dev, cur, s = torch.device("cpu"), None, None
        self._chol_local = False
        self.dev.prepare(A, snr_db, n_bits, quant_kind, thresholds, labels, stream=s)
        if not isinstance(self.shift, torch.Tensor) or self.shift.device != dev:
            self.shift = torch.empty(1, dtype=torch.float64, device=dev)
        if not self._guarded(self.dev.cconst_max, out=self.shift, stream=s):
            self.shift.fill_(float("inf"))  # the failure rides the shift as the kernel would have written it
        if cur is not None and s != cur.cuda_stream:  # the collective runs behind torch's current stream
            ev = torch.cuda.Event()
            ev.record(torch.cuda.ExternalStream(s, device=dev))
            cur.wait_event(ev)
        if self.world > 1:
            dist.all_reduce(self.shift, op=dist.ReduceOp.MAX, group=self.group)

    def _buf(self, key, shape, device):
        import torch
        b = self._bufs.get(key)
        if b is None or tuple(b.shape) != tuple(shape) or b.device != device:
            b = torch.empty(shape, dtype=torch.float64, device=device)
            self._bufs[key] = b
        return b

    def _guarded(self, fn, *a, **kw):
        """Run a device call of this rank; a Cholesky failure the library has already surfaced (it reports the
        deferred status at the first call that finds it complete) is recorded instead of raised, so every rank
        still reaches the step's collectives and all of them raise together at finish()."""
        if getattr(self, "_chol_local", False):
            return False
        try:
            fn(*a, **kw)
            return True
        except ValueError as e:
            if str(e) != _lib.CHOL_MESSAGE:
                raise
            self._chol_local = True
            return False

    def _chol_flag(self, device):
        import torch
        local = 1.0 if getattr(self, "_chol_local", False) else 0.0
        if isinstance(self.shift, torch.Tensor):
            return torch.clamp(torch.isinf(self.shift).to(torch.float64).reshape(1), min=local)
        return torch.tensor([1.0 if (local or math.isinf(float(self.shift))) else 0.0], dtype=torch.float64,
                            device=device)

    def estimate(self, y, chunks=None, scatter=True, sync=True, mode=_lib.MODE_ALL, param=0.0):
        """'all'-mode estimates of y (B, M) complex128 tensor.

        scatter=True: reduce-scatter per chunk, returns (rows, h) with h (n, N) complex128 the estimates of
        this rank's rows (global row indices `rows`, a LongTensor); scatter=False: all-reduce, every rank
        gets h for all B rows (rows = None).  The partial kernels run on torch's current stream, each
        chunk's collective asynchronously on RCCL's stream behind it.  sync=False: no host synchronisation; call
        finish() before reading h (rows whose shifted sum underflowed are NaN until then).  mode / param: the
        reference's selective modes (gmm_cplx_bussgang.py:197-219, :229-242) on the native path (comm=...)."""
        import torch
        import torch.distributed as dist
        if self.native is not None:
            return self._estimate_native(y, chunks, scatter, sync, mode, param)
        if mode != _lib.MODE_ALL:
            raise NotImplementedError("selective modes K-shard through the library's communicator (comm=...)")
        B = y.shape[0]
        W = 2 * self.N + 2
        dev = y.device
        stream = torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else None
        multi = self.world > 1
        use_rs = scatter and multi
        bounds = chunk_bounds(B, default_chunks(self.world) if chunks is None else chunks, self.world, use_rs)
        works, pieces = [], []
        for i, (lo, hi) in enumerate(bounds):
            n = hi - lo
            npad = -(-n // self.world) * self.world if use_rs else n
            pk = self._buf(("pk", i), (npad, W), dev)
            if npad > n:
                pk[n:].zero_()
            if not self._guarded(self.dev.partial_shifted, y[lo:hi], self.shift, out=pk[:n], stream=stream):
                pk[:n].zero_()
            if use_rs:
                out = self._buf(("rs", i), (npad // self.world, W), dev)
                works.append(dist.reduce_scatter_tensor(out, pk, op=dist.ReduceOp.SUM, group=self.group,
                                                        async_op=True))
                r0 = lo + self.rank * (npad // self.world)
                pieces.append((r0, min(hi, r0 + npad // self.world), out))
            else:
                if multi:
                    works.append(dist.all_reduce(pk[:n], op=dist.ReduceOp.SUM, group=self.group, async_op=True))
                pieces.append((lo, hi, pk[:n]))
        for wk in works:
            wk.wait()  # RCCL: the current stream waits on the collective (no host wait)
        rows = torch.cat([r[:max(0, b - a)] for a, b, r in pieces])
        # the step's flag word: [rows to recombine exactly, Cholesky failure on some rank], agreed with one MAX
        bad = rows[:, 0] < UNDERFLOW_S
        flags = torch.cat([bad.sum().to(torch.float64).reshape(1), self._chol_flag(dev)])
        if multi:
            dist.all_reduce(flags, op=dist.ReduceOp.MAX, group=self.group)
        if self._pending is not None:  # the step it supersedes can no longer be repaired: keep its flags apart
            prev = self._pending[5]
            self._flag_acc = prev if self._flag_acc is None else torch.maximum(self._flag_acc, prev)
        h = _packed_to_complex(rows)
        idx = torch.cat([torch.arange(a, max(a, b), device=dev) for a, b, _ in pieces]) if use_rs else None
        self._pending = (y, use_rs, bad, idx, h, flags)
        if sync:
            return self.finish()
        return idx, h

    def finish(self):
        """Read the flag words of the steps since the last finish() (one host sync): raise ValueError with the
        reference's message if a Cholesky factorisation failed on any rank, recombine the underflowed rows of the
        latest result exactly (in place) and return it as (rows, h)."""
        if self.native is not None:
            if self._native_rows is None:
                return None
            idx, h = self._native_rows
            self._native_rows = None
            import torch
            dev = torch.device("cuda", self.dev.device)
            self.native.finish(stream=torch.cuda.current_stream(dev).cuda_stream)
            return idx, h
        if self._pending is None:
            return None
        y, use_rs, bad, idx, h, flags = self._pending
        prev = self._flag_acc
        self._pending = self._flag_acc = None
        f_last = flags.tolist()
        f_prev = prev.tolist() if prev is not None else [0.0, 0.0]
        if f_last[1] > 0 or f_prev[1] > 0:
            raise ValueError(_lib.CHOL_MESSAGE)
        if f_prev[0] > 0:
            raise RuntimeError("an earlier K-shard estimate had rows whose shifted sum underflowed; estimate it "
                               "with sync=True to have them recombined")
        if f_last[0] > 0:
            self._repair(y, use_rs, bad, idx, h)
        return idx, h

    def _estimate_native(self, y, chunks, scatter, sync, mode, param):
        import torch
        ch = default_chunks(self.world) if chunks is None else chunks
        stream = torch.cuda.current_stream(y.device).cuda_stream
        ranges, h = self.native.estimate(y, mode, param, chunks=ch, scatter=scatter, stream=stream)
        idx = None
        if scatter:
            # the rows' global indices depend only on the layout: built once per layout, not per step (an arange and
            # a cat on the compute stream between two partial kernels)
            key = (tuple(ranges), y.device)
            idx = self._idx_cache.get(key) if self._idx_cache else None
            if idx is None:
                idx = torch.cat([torch.arange(a, b, device=y.device) for a, b in ranges]) if ranges else \
                    torch.empty(0, dtype=torch.int64, device=y.device)
                self._idx_cache = {key: idx}
        self._native_rows = (idx, h)
        if sync:
            return self.finish()
        return idx, h

    def _repair(self, y, use_rs, bad, idx, h):
        """Rare path: exact two-step combine (MAX of m, then SUM) of the unshifted FP64 partials, for the flagged
        rows only.  Under reduce-scatter every rank flags only rows it owns, so the row set is gathered first."""
        import torch
        import torch.distributed as dist
        dev = y.device
        stream = torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else None
        mine = torch.nonzero(bad, as_tuple=False).flatten()
        gmine = idx[mine] if use_rs else mine
        if use_rs:
            cnt = torch.tensor([gmine.numel()], dtype=torch.int64, device=dev)
            dist.all_reduce(cnt, op=dist.ReduceOp.MAX, group=self.group)
            padded = torch.full((int(cnt.item()),), -1, dtype=torch.int64, device=dev)
            padded[:gmine.numel()] = gmine
            allv = [torch.empty_like(padded) for _ in range(self.world)]
            dist.all_gather(allv, padded, group=self.group)
            grows = torch.unique(torch.cat(allv))
            grows = grows[grows >= 0]
        else:
            grows = gmine
        m, s, acc = self.dev.partial64(y[grows], stream=stream)
        if self.world > 1:
            hx = combine_partials_dist(m, s, acc, self.shift, self.N, self.group)
        else:
            hx = torch.from_numpy(combine_partials_numpy(
                [(m.cpu().numpy(), s.cpu().numpy(), acc.cpu().numpy())], self.N)).to(dev)
        if use_rs:  # this rank's flagged rows are a subset of grows (sorted): locate them
            pos = torch.searchsorted(grows, gmine)
            h[mine] = hx[pos]
        else:
            h[grows] = hx


def make_comm(rank, world, device=0, kind="rccl", group=None):
    """The libqce communicator of this rank.  kind "rccl": rank 0's ncclUniqueId is shared over the initialised
    torch.distributed group (any backend; gloo suffices), then every rank runs ncclCommInitRank on its device;
    kind "host": collectives through torch.distributed on host tensors (gloo), staged by the library."""
    import torch
    import torch.distributed as dist
    if kind == "rccl":
        obj = [_lib.Comm.unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(obj, src=0, group=group)
        return _lib.Comm(obj[0], rank, world, device)
    if kind != "host":
        raise ValueError(f"unknown communicator kind {kind!r}")

    def fn(op, send, recv):
        ts, tr = torch.from_numpy(send), torch.from_numpy(recv)
        if op in (_lib.COLL_ALLREDUCE_SUM, _lib.COLL_ALLREDUCE_MAX):
            tr.copy_(ts)
            dist.all_reduce(tr, op=dist.ReduceOp.SUM if op == _lib.COLL_ALLREDUCE_SUM else dist.ReduceOp.MAX,
                            group=group)
        elif op == _lib.COLL_REDUCE_SCATTER_SUM:
            tot = ts.clone()
            dist.all_reduce(tot, op=dist.ReduceOp.SUM, group=group)  # gloo has no reduce_scatter
            n = tr.numel()
            tr.copy_(tot[rank * n:(rank + 1) * n])
        elif op == _lib.COLL_ALLGATHER:
            dist.all_gather(list(tr.chunk(world)), ts, group=group)
        else:
            raise ValueError(op)
    return _lib.Comm.host(rank, world, device, fn)


class BatchShardEstimator:
    """Batch-sharded replicas: the full mixture on every GPU, a disjoint slice of y per rank."""

    def __init__(self, means_cplx, covs_cplx, weights, device=0, precision="f64"):
        self.dev = _lib.DeviceModel(means_cplx, covs_cplx, weights, device=device)
        if precision != "f64":
            self.dev.set_precision(precision)

    def prepare(self, *args, **kw):
        self.dev.prepare(*args, **kw)

    def estimate(self, y_local, mode=_lib.MODE_ALL, param=0.0, out=None, stream=None):
        return self.dev.estimate(y_local, mode, param, out=out, stream=stream)
