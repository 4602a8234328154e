"""Multi-GPU decomposition of the estimate path (one process per GPU, torch.distributed).

Two ways to split one SNR point's work:

* **batch shards** (``BatchShardEstimator``): every rank holds the whole mixture and estimates a
  disjoint slice of the observations.  No data-path collective — the samples are independent.
* **component shards** (``ComponentShardEstimator``): rank g holds components K_g and returns, per
  sample, the running max m_g, s_g = sum_{k in K_g} e^{lp_k - m_g} and
  acc_g = sum_{k in K_g} e^{lp_k - m_g} (W_k y + b_k) (``qce_estimate_partial``).  With the
  y-independent shift M* = max_k c_k >= lp_k (c_k = log w_k + 2 log det P_k - M log pi, known after
  prepare; one scalar MAX all-reduce per SNR) every rank rescales to s'_g = s_g e^{m_g - M*},
  acc'_g = acc_g e^{m_g - M*} in FP64 and ONE SUM all-reduce of the packed (B, 2N+1) buffer gives
  h = acc / s.  Rows whose s underflows everywhere (all quad forms > ~700) are recombined with a
  MAX all-reduce of m first.
"""
import numpy as np

from . import _lib


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
    """Distributed combine of one rank's partial (torch tensors on this rank's device).

    m, s: (B,) float64; acc: (B, 2N) float32; shift: the global M* (python float).
    Returns h (B, N) complex128 on every rank.  One SUM all-reduce on the data path."""
    import torch
    import torch.distributed as dist
    B = m.shape[0]
    buf = torch.empty((B, 2 * N + 1), dtype=torch.float64, device=m.device)
    sc = torch.exp(m - shift)
    buf[:, 0] = s * sc
    buf[:, 1:] = acc.to(torch.float64) * sc[:, None]
    dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    bad = buf[:, 0] == 0
    nbad = bad.sum()
    dist.all_reduce(nbad, op=dist.ReduceOp.MAX, group=group)  # tiny: agree on the fallback
    if int(nbad.item()) > 0:
        idx = torch.nonzero(bad, as_tuple=False).flatten()
        # underflow guard: exact two-step combine for the affected rows
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


class ComponentShardEstimator:
    """K-sharded 'all'-mode estimator: this rank's slice of the mixture on its own GPU."""

    def __init__(self, means_cplx, covs_cplx, weights, rank, world, device=0, group=None):
        K = np.asarray(covs_cplx).shape[0]
        self.lo, self.hi = component_slices(K, world)[rank]
        sl = slice(self.lo, self.hi)
        means = None if means_cplx is None else np.asarray(means_cplx)[sl]
        self.dev = _lib.DeviceModel(means, np.asarray(covs_cplx)[sl], np.asarray(weights)[sl], device=device)
        self.N = self.dev.N
        self.group = group
        self.shift = None

    def prepare(self, A, snr_db, n_bits, quant_kind=_lib.QUANT_UNIFORM, thresholds=None, labels=None, stream=None):
        import torch
        import torch.distributed as dist
        self.dev.prepare(A, snr_db, n_bits, quant_kind, thresholds, labels, stream=stream)
        c = self.dev.tables()["cconst"]
        dev = torch.device("cuda", self.dev.device) if torch.cuda.is_available() else torch.device("cpu")
        t = torch.tensor([float(np.max(c))], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        self.shift = float(t.item())

    def estimate(self, y, stream=None):
        m, s, acc = self.dev.partial(y, stream=stream)
        return combine_partials_dist(m, s, acc, self.shift, self.N, self.group)


class BatchShardEstimator:
    """Batch-sharded replicas: the full mixture on every GPU, a disjoint slice of y per rank."""

    def __init__(self, means_cplx, covs_cplx, weights, device=0):
        self.dev = _lib.DeviceModel(means_cplx, covs_cplx, weights, device=device)

    def prepare(self, *args, **kw):
        self.dev.prepare(*args, **kw)

    def estimate(self, y_local, mode=_lib.MODE_ALL, param=0.0, out=None, stream=None):
        return self.dev.estimate(y_local, mode, param, out=out, stream=stream)
