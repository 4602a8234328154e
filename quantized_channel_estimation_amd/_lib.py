"""ctypes binding of libqce.so (include/qce.h).

The library is the only compute path: if it is missing or no HIP device is visible, every
estimator call raises — there is no CPU fallback in this package.
"""
import atexit
import ctypes
import os
import threading
import weakref

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("QCE_LIB") or os.path.join(_PKG, "libqce.so")  # QCE_LIB: diagnostic builds only

QCE_OK, QCE_EARG, QCE_ECHOL, QCE_ENOTIMPL, QCE_EHIP, QCE_ESTATE, QCE_ECOMM = range(7)
MODE_ALL, MODE_TOPN, MODE_CUMP = 0, 1, 2
OPT_BETA_FIRST = 1
OPT_PRECISION = 2
OPT_RESERVE_CUS = 3
PRECISION_F64, PRECISION_FAST = 0, 1
QUANT_UNIFORM, QUANT_LLOYD, QUANT_OTHER = 0, 1, 2
IO_HOST, IO_DEVICE = 0, 1
COMM_ID_BYTES = 128
COMM_RCCL, COMM_HOST = 0, 1
COLL_ALLREDUCE_SUM, COLL_ALLREDUCE_MAX, COLL_REDUCE_SCATTER_SUM, COLL_ALLGATHER = range(4)

# The reference's message for a non-positive-definite Cr_k (gmm_cplx_bussgang.py:33-37, raised at :43-46); the
# library returns the same text with QCE_ECHOL (csrc/qce_capi.hip check_status), the K-shard path raises it from
# the flag its shift carries (sharding.py).
CHOL_MESSAGE = ("Fitting the mixture model failed because some components have ill-defined empirical covariance "
                "(for instance caused by singleton or collapsed samples). Try to decrease the number of "
                "components, or increase reg_covar.")

_c_dbl_p = ctypes.POINTER(ctypes.c_double)
_c_flt_p = ctypes.POINTER(ctypes.c_float)
_c_i64_p = ctypes.POINTER(ctypes.c_int64)
_vp = ctypes.c_void_p

# name -> (restype, argtypes); every symbol include/qce.h declares
SIGNATURES = {
    "qce_version": (ctypes.c_int, []),
    "qce_build_id": (ctypes.c_char_p, []),
    "qce_last_error": (ctypes.c_char_p, []),
    "qce_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "qce_model_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _vp, _vp, _vp, ctypes.c_int,
                                        ctypes.POINTER(_vp)]),
    "qce_model_destroy": (ctypes.c_int, [_vp]),
    "qce_model_set_params": (ctypes.c_int, [_vp, _vp, _vp, _vp]),
    "qce_em_toeplitz": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int, _vp, ctypes.c_int, _vp, ctypes.c_double,
                                       ctypes.c_int, _vp, ctypes.c_int, _vp]),
    "qce_scm_generate": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, _vp,
                                        _vp, _vp, ctypes.c_uint64, _vp, _vp, ctypes.c_int, ctypes.c_int, _vp]),
    "qce_rate_mf": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int, _vp, _vp, _vp, ctypes.c_int, ctypes.c_int,
                                   _vp]),
    "qce_rate_bound": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int, _vp, _vp, ctypes.c_double, _vp,
                                      ctypes.c_int, ctypes.c_int, _vp]),
    "qce_model_set_option": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_double]),
    "qce_estimate_assigned": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp, _vp, ctypes.c_int, _vp]),
    "qce_estimate_ls": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp, _vp, ctypes.c_int, _vp]),
    "qce_estimate_ls_general": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp, _vp, ctypes.c_int, _vp]),
    "qce_prepare": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_int, _vp, _vp,
                                   ctypes.c_int, _vp]),
    "qce_estimate": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int, ctypes.c_double, _vp, ctypes.c_int, _vp]),
    "qce_log_prob": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp, _vp, _vp, ctypes.c_int, _vp]),
    "qce_estimate_partial": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp, _vp, _vp, ctypes.c_int, _vp]),
    "qce_estimate_partial_f64": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp, _vp, _vp, ctypes.c_int, _vp]),
    "qce_estimate_partial_shifted": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp, _vp, ctypes.c_int, _vp]),
    "qce_cconst_max": (ctypes.c_int, [_vp, _vp, ctypes.c_int, _vp]),
    "qce_get_tables": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "qce_model_info": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                      ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "qce_synchronize": (ctypes.c_int, [_vp]),
    "qce_model_kernel": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int)]),
    "qce_host_alloc": (ctypes.c_int, [ctypes.c_size_t, ctypes.POINTER(_vp)]),
    "qce_host_free": (ctypes.c_int, [_vp]),
    "qce_observe": (ctypes.c_int, [_vp, ctypes.c_int64, ctypes.c_int, _vp, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                   _vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_double, _vp, _vp, ctypes.c_int, _vp,
                                   ctypes.c_int, ctypes.c_int, _vp]),
    "qce_sq_error": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp, ctypes.c_int, ctypes.c_int, _vp]),
    "qce_em_estep": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp, _vp, ctypes.c_int, _vp]),
    "qce_em_mstep": (ctypes.c_int, [_vp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, _vp, ctypes.c_double,
                                    ctypes.c_int, ctypes.c_int, _vp, _vp, _vp, ctypes.c_int, ctypes.c_int, _vp]),
    "qce_model_structure": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                           ctypes.POINTER(ctypes.c_int)]),
    # K-shard over a communicator (csrc/qce_kshard.hip)
    "qce_comm_unique_id": (ctypes.c_int, [_vp]),
    "qce_comm_init": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_vp)]),
    "qce_comm_init_host": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, _vp, ctypes.POINTER(_vp)]),
    "qce_comm_destroy": (ctypes.c_int, [_vp]),
    "qce_comm_info": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                     ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "qce_kshard_slice": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                        ctypes.POINTER(ctypes.c_int)]),
    "qce_kshard_rows": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp,
                                       ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    "qce_kshard_create": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.POINTER(_vp)]),
    "qce_kshard_destroy": (ctypes.c_int, [_vp]),
    "qce_kshard_set_spare": (ctypes.c_int, [_vp, _vp]),
    "qce_kshard_prepare": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_int, _vp,
                                          _vp, ctypes.c_int, _vp]),
    "qce_kshard_estimate": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                           ctypes.c_int, _vp, _vp]),
    "qce_kshard_finish": (ctypes.c_int, [_vp, _vp]),
    "qce_kshard_timing": (ctypes.c_int, [_vp, ctypes.c_int]),
    "qce_kshard_kernel_ms": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]),
    "qce_kshard_flags": (ctypes.c_int, [_vp, _vp]),
}

# qce_host_collective: int (*)(void* user, int op, const double* send, double* recv, int64_t count)
HOST_COLLECTIVE = ctypes.CFUNCTYPE(ctypes.c_int, _vp, ctypes.c_int, _c_dbl_p, _c_dbl_p, ctypes.c_int64)

_lib = None


class QceError(RuntimeError):
    pass


def load():
    """Load libqce.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `python -m quantized_channel_estimation_amd.build`"
                          " (there is no CPU fallback)")
    # One HIP runtime per process: torch ships its own libamdhip64 (SONAME libamdhip64.so.7, loaded
    # from torch/lib as "libamdhip64.so").  Loading torch first makes libqce.so's NEEDED
    # libamdhip64.so.7 bind to that same runtime; the other order leaves two HIP/HSA runtimes in
    # the process and torch then reports no GPU.
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is part of the image
        pass
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc):
    """Map a status code to the reference's exception types."""
    if rc == QCE_OK:
        return
    msg = load().qce_last_error().decode("utf-8", "replace")
    if rc in (QCE_EARG, QCE_ECHOL):
        raise ValueError(msg)
    if rc == QCE_ENOTIMPL:
        raise NotImplementedError(msg)
    raise QceError(f"[qce status {rc}] {msg}")


# Every live handle of this process (DeviceModel, Comm, KShard), closed in dependency order by an atexit hook while the
# HIP runtime and RCCL are still fully up: objects Python never collects (reference cycles, module
# globals) otherwise reach their teardown only through the runtimes' own exit-time destructors.
_live = {"kshard": weakref.WeakSet(), "comm": weakref.WeakSet(), "model": weakref.WeakSet()}


def _close_all_at_exit():
    if os.environ.get("QCE_NO_EXIT_CLOSE") == "1":  # diagnostic: leave teardown to the runtimes' destructors
        return
    for kind in ("kshard", "model", "comm"):
        for obj in list(_live[kind]):
            try:
                obj.close()
            except Exception:
                pass


atexit.register(_close_all_at_exit)


def build_id():
    """Source digest the loaded libqce.so was built from (qce_build_id)."""
    return load().qce_build_id().decode()


def check_build_current():
    """Raise if the loaded library was not built from the sources in this tree (a stale libqce.so)."""
    from . import build as _b
    if not os.path.isdir(_b.CSRC):
        return
    want, have = _b.source_digest(), build_id()
    if have.split("-")[0] != want:
        raise QceError(f"{LIB_PATH} was built from sources {have}, the tree has {want}: rebuild it")


def device_count():
    n = ctypes.c_int(0)
    check(load().qce_device_count(ctypes.byref(n)))
    return n.value


def ptr(a):
    """Data pointer of a contiguous numpy array or torch tensor (None -> NULL)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        if not a.flags["C_CONTIGUOUS"]:
            raise ValueError("array must be C-contiguous")
        return a.ctypes.data
    return a.data_ptr()


class _PinnedBlock:
    """A page-locked host allocation (qce_host_alloc); returned to the pool when the last array on it is gone."""

    def __init__(self, nbytes):
        p = _vp()
        check(load().qce_host_alloc(int(nbytes), ctypes.byref(p)))
        self.ptr, self.nbytes = p.value, int(nbytes)

    def __del__(self):
        try:
            _pinned_pool.give_back(self)
        except Exception:
            pass


class _PinnedPool:
    """Free page-locked blocks kept for reuse (the drop-in numpy API's result arrays): the estimate's D2H lands in
    them directly, and a block the caller dropped serves the next call without new page faults.  At most
    `cap_bytes` of free blocks are kept; the rest are freed.  Thread-safe: an array dropped on another
    thread returns its block while take() searches, so the search and the removal are one critical section and the
    block handed out is checked against the request."""

    def __init__(self, cap_bytes=1 << 30):
        self.cap = cap_bytes
        self.free = []  # (ptr, nbytes) records of blocks not referenced by any array
        self.lock = threading.Lock()

    def take(self, nbytes):
        nbytes = int(nbytes)
        with self.lock:
            best = None
            for rec in self.free:
                if nbytes <= rec[1] <= 2 * nbytes and (best is None or rec[1] < best[1]):
                    best = rec
            if best is not None:
                self.free.remove(best)  # by identity of the record, inside the lock
        if best is not None:
            p, n = best
            if n < nbytes:  # pragma: no cover - guarded above; never hand out a block the D2H would overrun
                raise QceError(f"pinned pool block of {n} bytes for a request of {nbytes}")
            blk = _PinnedBlock.__new__(_PinnedBlock)
            blk.ptr, blk.nbytes = p, n
            return blk
        return _PinnedBlock(nbytes)

    def give_back(self, blk):
        to_free = []
        with self.lock:
            if blk.ptr is None:
                return
            self.free.append((blk.ptr, blk.nbytes))
            blk.ptr = None
            while sum(n for _, n in self.free) > self.cap:
                to_free.append(self.free.pop(0)[0])
        for p in to_free:
            load().qce_host_free(p)


_pinned_pool = _PinnedPool()


class _PinnedArrayBase:
    def __init__(self, blk, shape, dtype):
        self.blk = blk
        self.__array_interface__ = {"shape": tuple(shape), "typestr": np.dtype(dtype).str,
                                    "data": (blk.ptr, False), "version": 3}


# results at least this large come from the pinned pool (the size from which QCE_IO_HOST pipelines, 2 x 4096 rows of
# a 64-wide row); smaller ones are ordinary numpy arrays
PINNED_MIN_BYTES = 8 << 20


def host_empty(shape, dtype=np.complex128):
    """np.empty((shape), dtype) in page-locked memory from the pool (ordinary numpy array semantics; the block goes
    back to the pool when the array and its views are gone)."""
    nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
    if nbytes < PINNED_MIN_BYTES or os.environ.get("QCE_PINNED_RESULTS", "1") == "0":
        return np.empty(shape, dtype=dtype)
    return np.asarray(_PinnedArrayBase(_pinned_pool.take(nbytes), shape, dtype))


class DeviceModel:
    """Owner of one qce_model handle (device tables of one Gaussian mixture on one GPU)."""

    def __init__(self, means_cplx, covs_cplx, weights, device=0):
        lib = load()
        covs = np.ascontiguousarray(covs_cplx, dtype=np.complex128)
        K, N = covs.shape[0], covs.shape[-1]
        means = None if means_cplx is None else np.ascontiguousarray(means_cplx, dtype=np.complex128).reshape(K, N)
        w = np.ascontiguousarray(weights, dtype=np.float64).reshape(K)
        h = _vp()
        check(lib.qce_model_create(K, N, ptr(means), ptr(covs), ptr(w), int(device), ctypes.byref(h)))
        self._h = h
        _live["model"].add(self)
        self.K, self.N, self.device = K, N, int(device)
        self.M = 0
        self.precision = "f64"
        self.has_mean = bool(means is not None and np.any(means != 0))

    @property
    def handle(self):
        return self._h

    def set_params(self, means_cplx, covs_cplx, weights):
        """Same K, N; new parameters (prepared state dropped)."""
        covs = np.ascontiguousarray(covs_cplx, dtype=np.complex128)
        if covs.shape != (self.K, self.N, self.N):
            raise ValueError(f"covariances must be ({self.K}, {self.N}, {self.N})")
        means = None if means_cplx is None else np.ascontiguousarray(means_cplx, dtype=np.complex128).reshape(
            self.K, self.N)
        w = np.ascontiguousarray(weights, dtype=np.float64).reshape(self.K)
        check(load().qce_model_set_params(self._h, ptr(means), ptr(covs), ptr(w)))
        self.M = 0
        self.has_mean = bool(means is not None and np.any(means != 0))

    def close(self):
        if getattr(self, "_h", None):
            load().qce_model_destroy(self._h)
            self._h = None
            _live["model"].discard(self)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def prepare(self, A, snr_db, n_bits, quant_kind=QUANT_UNIFORM, thresholds=None, labels=None, stream=None):
        lib = load()
        if A is None:
            M, a = self.N, None
        else:
            a = np.ascontiguousarray(A, dtype=np.complex128)
            if a.ndim != 2 or a.shape[1] != self.N:
                raise ValueError(f"A must be (M, {self.N}), got {a.shape}")
            M = a.shape[0]
        thr = lab = None
        nlev = 0
        if labels is not None:
            lab = np.ascontiguousarray(labels, dtype=np.float64)
            thr = np.ascontiguousarray(thresholds, dtype=np.float64)
            nlev = lab.size
        check(lib.qce_prepare(self._h, ptr(a), int(M), float(snr_db), float(n_bits), int(quant_kind), ptr(thr),
                              ptr(lab), int(nlev), stream))
        self.M = M

    def estimate(self, y, mode=MODE_ALL, param=0.0, out=None, stream=None):
        """y: (B,M) complex128 numpy array (host) or torch.complex128 CUDA tensor (device)."""
        io = IO_HOST if isinstance(y, np.ndarray) else IO_DEVICE
        B = y.shape[0]
        if io == IO_HOST:
            y = np.ascontiguousarray(y, dtype=np.complex128)
            if out is None:
                out = host_empty((B, self.N), np.complex128)  # the D2H lands in it directly
        elif out is None:
            import torch
            out = torch.empty((B, self.N), dtype=torch.complex128, device=y.device)
        if y.shape[1] != self.M:
            raise ValueError(f"y must have {self.M} columns, got {y.shape[1]}")
        self._order_before(y, io, stream)
        check(load().qce_estimate(self._h, ptr(y), int(B), int(mode), float(param), ptr(out), io, stream))
        self._order_after(io, stream)
        return out

    @staticmethod
    def _order_before(y, io, stream):
        """... and the inputs torch produced on its current stream must be complete before that stream runs."""
        if io == IO_DEVICE and not stream:
            import torch
            torch.cuda.current_stream(y.device).synchronize()

    def _order_after(self, io, stream):
        """Device I/O without an explicit stream ran on the model's own non-blocking stream (a NULL
        handle there means "the model's stream"): finish it so torch's streams see the results."""
        if io == IO_DEVICE and not stream:
            self.synchronize()

    def log_prob(self, X, want_lp=True, want_proba=False, want_labels=False):
        X = np.ascontiguousarray(X, dtype=np.complex128)
        B = X.shape[0]
        if X.ndim != 2 or X.shape[1] != self.M:
            raise ValueError(f"X must be (B, {self.M}), got {X.shape}")
        lp = np.empty((B, self.K)) if want_lp else None
        pr = np.empty((B, self.K)) if want_proba else None
        lb = np.empty(B, dtype=np.int64) if want_labels else None
        check(load().qce_log_prob(self._h, ptr(X), int(B), ptr(lp), ptr(pr), ptr(lb), IO_HOST, None))
        return lp, pr, lb

    def partial(self, y, m_out=None, s_out=None, acc_out=None, stream=None):
        io = IO_HOST if isinstance(y, np.ndarray) else IO_DEVICE
        B = y.shape[0]
        if io == IO_HOST:
            y = np.ascontiguousarray(y, dtype=np.complex128)
            m_out = np.empty(B) if m_out is None else m_out
            s_out = np.empty(B) if s_out is None else s_out
            acc_out = np.empty((B, 2 * self.N), dtype=np.float32) if acc_out is None else acc_out
        else:
            import torch
            dev = y.device
            m_out = torch.empty(B, dtype=torch.float64, device=dev) if m_out is None else m_out
            s_out = torch.empty(B, dtype=torch.float64, device=dev) if s_out is None else s_out
            acc_out = torch.empty((B, 2 * self.N), dtype=torch.float32, device=dev) if acc_out is None else acc_out
        self._order_before(y, io, stream)
        check(load().qce_estimate_partial(self._h, ptr(y), int(B), ptr(m_out), ptr(s_out), ptr(acc_out), io, stream))
        self._order_after(io, stream)
        return m_out, s_out, acc_out

    def partial64(self, y, m_out=None, s_out=None, acc_out=None, stream=None):
        """K-shard partial with an FP64 accumulator (qce_estimate_partial_f64): (m, s, acc (B, 2N) f64)."""
        io = IO_HOST if isinstance(y, np.ndarray) else IO_DEVICE
        B = y.shape[0]
        if io == IO_HOST:
            y = np.ascontiguousarray(y, dtype=np.complex128)
            m_out = np.empty(B) if m_out is None else m_out
            s_out = np.empty(B) if s_out is None else s_out
            acc_out = np.empty((B, 2 * self.N)) if acc_out is None else acc_out
        else:
            import torch
            dev = y.device
            m_out = torch.empty(B, dtype=torch.float64, device=dev) if m_out is None else m_out
            s_out = torch.empty(B, dtype=torch.float64, device=dev) if s_out is None else s_out
            acc_out = torch.empty((B, 2 * self.N), dtype=torch.float64, device=dev) if acc_out is None else acc_out
        self._order_before(y, io, stream)
        check(load().qce_estimate_partial_f64(self._h, ptr(y), int(B), ptr(m_out), ptr(s_out), ptr(acc_out), io,
                                              stream))
        self._order_after(io, stream)
        return m_out, s_out, acc_out

    def partial_shifted(self, y, shift, out=None, stream=None):
        """Shifted packed K-shard partial (qce_estimate_partial_shifted): (B, 2N+2) f64 rows
        [s e^{m-shift}, 0, acc e^{m-shift}] that sum over shards.  shift: a float (host I/O) or a one-element
        float64 tensor on the device (device I/O, no host round trip)."""
        io = IO_HOST if isinstance(y, np.ndarray) else IO_DEVICE
        B = y.shape[0]
        if io == IO_HOST:
            y = np.ascontiguousarray(y, dtype=np.complex128)
            out = np.empty((B, 2 * self.N + 2)) if out is None else out
            sh = np.array([float(shift)])
        else:
            import torch
            if out is None:
                out = torch.empty((B, 2 * self.N + 2), dtype=torch.float64, device=y.device)
            sh = shift if isinstance(shift, torch.Tensor) else torch.tensor([float(shift)], dtype=torch.float64,
                                                                             device=y.device)
        self._order_before(y, io, stream)
        check(load().qce_estimate_partial_shifted(self._h, ptr(y), int(B), ptr(sh), ptr(out), io, stream))
        self._order_after(io, stream)
        return out

    def cconst_max(self, out=None, stream=None):
        """max_k c_k of the last prepare: a float, or written into the one-element device tensor `out`
        (asynchronously on `stream`)."""
        if out is None:
            v = np.empty(1)
            check(load().qce_cconst_max(self._h, ptr(v), IO_HOST, None))
            return float(v[0])
        check(load().qce_cconst_max(self._h, ptr(out), IO_DEVICE, stream))
        return out

    def cconst(self):
        """c_k = -M log(pi) + 2 log det P_k + log w_k of the last prepare (K,) — the shard shift input."""
        c = np.empty(self.K)
        check(load().qce_get_tables(self._h, None, None, None, None, None, None, None, ptr(c)))
        return c

    def set_precision(self, precision):
        """'f64' (default: the reference's complex128 arithmetic) or 'fast' (fp16 two-term split products,
        fp32 accumulation) for the dense 'all' mode and the K-shard partial."""
        val = {"f64": PRECISION_F64, "fast": PRECISION_FAST}[precision]
        self.set_option(OPT_PRECISION, val)
        self.precision = precision

    def reserve_cus(self, n):
        """CUs the persistent estimate kernels leave free for a concurrent communication stream (QCE_OPT_RESERVE_CUS;
        the prepared tables stay valid)."""
        check(load().qce_model_set_option(self._h, OPT_RESERVE_CUS, float(n)))

    def set_option(self, option, value):
        check(load().qce_model_set_option(self._h, int(option), float(value)))
        self.M = 0

    def estimate_assigned(self, y, comp=None, ls=False):
        """h_b = W_c y_b + b_c (ls: the least-squares solution with A_eff_c; ls="general": full-column-rank A_eff_c, not only
        column-orthogonal ones), c = comp[b] (None: c = b);
        host numpy I/O."""
        y = np.ascontiguousarray(y, dtype=np.complex128)
        B = y.shape[0]
        if y.ndim != 2 or y.shape[1] != self.M:
            raise ValueError(f"y must be (B, {self.M})")
        c = None if comp is None else np.ascontiguousarray(comp, dtype=np.int64).reshape(B)
        out = np.empty((B, self.N), dtype=np.complex128)
        if ls == "general":
            fn = load().qce_estimate_ls_general
        else:
            fn = load().qce_estimate_ls if ls else load().qce_estimate_assigned
        check(fn(self._h, ptr(y), int(B), ptr(c), ptr(out), IO_HOST, None))
        return out

    _TABLES = ("means_y", "Cy", "Cr", "P", "A_eff", "W", "b", "cconst")

    def tables(self, names=None):
        """Per-SNR tables of the last prepare (qce_get_tables); `names` restricts the copy."""
        K, M, N = self.K, self.M, self.N
        shapes = dict(means_y=(K, M), Cy=(K, M, M), Cr=(K, M, M), P=(K, M, M), A_eff=(K, M, N), W=(K, N, M),
                      b=(K, N), cconst=(K,))
        names = self._TABLES if names is None else tuple(names)
        t = {k: np.empty(shapes[k], float if k == "cconst" else complex) for k in names}
        check(load().qce_get_tables(self._h, *(ptr(t.get(k)) for k in self._TABLES)))
        return t

    def synchronize(self):
        check(load().qce_synchronize(self._h))

    KERNELS = {0: "none", 1: "f64_4m", 2: "f64_3m", 3: "f64_wide", 4: "big", 5: "fourier", 6: "fast"}

    def kernel(self):
        """'all'-mode kernel family of the last prepare (qce_model_kernel): f64_3m, f64_4m, fourier, ..."""
        k = ctypes.c_int()
        check(load().qce_model_kernel(self._h, ctypes.byref(k)))
        return self.KERNELS[k.value]

    def structure(self):
        """(n1, n2, fourier_active): block-circulant structure found at creation ((0, 0) if none) and
        whether the last prepare took the Fourier-domain path (qce_fft.hip)."""
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(load().qce_model_structure(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, c.value


def kshard_slice(K, world, rank):
    """Components [lo, hi) of `rank` in the library's balanced contiguous split (qce_kshard_slice)."""
    lo, hi = ctypes.c_int(), ctypes.c_int()
    check(load().qce_kshard_slice(int(K), int(world), int(rank), ctypes.byref(lo), ctypes.byref(hi)))
    return lo.value, hi.value


def kshard_layout(world, rank):
    """(world, rank) a K-shard's rows are laid out for: the communicator's, or on a world-1 communicator the test hook
    QCE_KSHARD_EMULATE_WORLD="W[:R]" (one GPU rehearsing rank R of a W-GPU step; csrc/qce_kshard.hip)."""
    e = os.environ.get("QCE_KSHARD_EMULATE_WORLD", "")
    if world != 1 or not e:
        return world, rank
    try:
        w, _, r = e.partition(":")
        w, r = int(w), int(r or 0)
    except ValueError:
        return world, rank
    if w < 2 or w > 4096 or not 0 <= r < w:
        return world, rank
    return w, r


def kshard_rows(B, chunks, world, rank, scatter):
    """Global row ranges [(r0, r1), ...] of the rows a rank's qce_kshard_estimate writes, in h_out order."""
    cap = max(1, int(chunks)) + 1
    arr = np.empty(2 * cap, dtype=np.int64)
    n = ctypes.c_int()
    check(load().qce_kshard_rows(int(B), int(chunks), int(world), int(rank), int(bool(scatter)), ptr(arr), cap,
                                 ctypes.byref(n)))
    return [(int(arr[2 * i]), int(arr[2 * i + 1])) for i in range(n.value)]


class Comm:
    """A libqce communicator (qce_comm): RCCL (``Comm(uid, rank, world, device)``, the uid from ``Comm.unique_id()``
    on one rank) or a host transport (``Comm.host(rank, world, device, fn)`` with fn(op, send, recv) on numpy
    float64 arrays, e.g. torch.distributed over gloo)."""

    @staticmethod
    def unique_id():
        buf = ctypes.create_string_buffer(COMM_ID_BYTES)
        check(load().qce_comm_unique_id(ctypes.cast(buf, _vp)))
        return buf.raw

    def __init__(self, uid, rank, world, device=0):
        if len(uid) != COMM_ID_BYTES:
            raise ValueError(f"unique id must be {COMM_ID_BYTES} bytes")
        buf = ctypes.create_string_buffer(bytes(uid), COMM_ID_BYTES)
        h = _vp()
        check(load().qce_comm_init(ctypes.cast(buf, _vp), int(rank), int(world), int(device), ctypes.byref(h)))
        self._h, self._cb = h, None
        self.rank, self.world, self.device, self.kind = int(rank), int(world), int(device), COMM_RCCL
        _live["comm"].add(self)

    @classmethod
    def host(cls, rank, world, device, fn):
        """fn(op, send, recv) -> None with send / recv numpy float64 views (QCE_COLL_* semantics, include/qce.h)."""
        self = cls.__new__(cls)
        world = int(world)

        def tramp(_user, op, send, recv, count):
            try:
                ns = count * world if op == COLL_REDUCE_SCATTER_SUM else count
                nr = count * world if op == COLL_ALLGATHER else count
                fn(op, np.ctypeslib.as_array(send, shape=(ns,)), np.ctypeslib.as_array(recv, shape=(nr,)))
                return 0
            except Exception:  # pragma: no cover - surfaces as QCE_ECOMM
                import traceback
                traceback.print_exc()
                return 1
        self._cb = HOST_COLLECTIVE(tramp)
        h = _vp()
        check(load().qce_comm_init_host(int(rank), world, int(device), ctypes.cast(self._cb, _vp), None,
                                        ctypes.byref(h)))
        self._h = h
        self.rank, self.world, self.device, self.kind = int(rank), world, int(device), COMM_HOST
        _live["comm"].add(self)
        return self

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None):
            load().qce_comm_destroy(self._h)
            self._h = None
            _live["comm"].discard(self)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class KShard:
    """qce_kshard: the K-shard estimator of one rank over a Comm; `model` is the DeviceModel of this rank's
    components kshard_slice(K, world, rank)."""

    def __init__(self, model, comm, K_total):
        h = _vp()
        check(load().qce_kshard_create(model.handle, comm.handle, int(K_total), ctypes.byref(h)))
        self._h, self.model, self.comm, self.K = h, model, comm, int(K_total)
        self._keep = None
        self._own = None  # private torch stream standing in for torch's null stream (_stream)
        self.layout_world, self.layout_rank = kshard_layout(comm.world, comm.rank)
        _live["kshard"].add(self)

    def _stream(self, stream):
        """(handle, torch's current stream) of the stream a K-shard call runs on: the caller's, else torch's current
        stream.  A null handle would mean "the model's own stream" to the library -- unordered with torch's work (y
        uploaded on the null stream could still be in flight) -- so torch's null stream is replaced by a private torch
        stream that waits for it."""
        import torch
        dev = torch.device("cuda", self.model.device)
        cur = torch.cuda.current_stream(dev)
        s = int(stream) if stream else cur.cuda_stream
        if s == 0:
            if self._own is None:
                self._own = torch.cuda.Stream(dev)
            self._own.wait_stream(cur)
            s = self._own.cuda_stream
        return s, cur

    def set_spare(self, spare):
        """Double-buffered tables: `spare` another DeviceModel of the same shard (qce_kshard_set_spare)."""
        check(load().qce_kshard_set_spare(self._h, spare.handle))
        self.spare = spare

    def close(self):
        if getattr(self, "_h", None):
            load().qce_kshard_destroy(self._h)
            self._h = None
            self._keep = None
            _live["kshard"].discard(self)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def prepare(self, A, snr_db, n_bits, quant_kind=QUANT_UNIFORM, thresholds=None, labels=None, stream=None):
        m = self.model
        if A is None:
            M, a = m.N, None
        else:
            a = np.ascontiguousarray(A, dtype=np.complex128)
            if a.ndim != 2 or a.shape[1] != m.N:
                raise ValueError(f"A must be (M, {m.N}), got {a.shape}")
            M = a.shape[0]
        thr = lab = None
        nlev = 0
        if labels is not None:
            lab = np.ascontiguousarray(labels, dtype=np.float64)
            thr = np.ascontiguousarray(thresholds, dtype=np.float64)
            nlev = lab.size
        stream, _ = self._stream(stream)
        check(load().qce_kshard_prepare(self._h, ptr(a), int(M), float(snr_db), float(n_bits), int(quant_kind),
                                        ptr(thr), ptr(lab), int(nlev), stream))
        m.M = M

    def estimate(self, y, mode=MODE_ALL, param=0.0, chunks=2, scatter=True, out=None, stream=None):
        """y (B, M) complex128 CUDA tensor (the same on every rank) -> (rows, h): h the estimates of the global rows
        `rows` (a list of (r0, r1) ranges in h's row order).  Asynchronous on `stream` (default: torch's current
        stream of y's device, see _stream); finish() is the sync point."""
        import torch
        B = y.shape[0]
        stream, cur = self._stream(stream)
        ch = int(chunks) if mode == MODE_ALL else 1
        rows = kshard_rows(B, ch, self.layout_world, self.layout_rank, scatter)
        n = sum(b - a for a, b in rows)
        if out is None:
            out = torch.empty((n, self.model.N), dtype=torch.complex128, device=y.device)
        elif tuple(out.shape) != (n, self.model.N):
            raise ValueError(f"out must be ({n}, {self.model.N})")
        if y.shape[1] != self.model.M:
            raise ValueError(f"y must have {self.model.M} columns, got {y.shape[1]}")
        check(load().qce_kshard_estimate(self._h, ptr(y), int(B), int(mode), float(param), ch, int(bool(scatter)),
                                         ptr(out), stream))
        # y and h of the steps whose collectives / row finalisation may still run on the library's communication
        # stream stay alive: the last two (step t+2 waits on the compute stream for step t's communication-stream work,
        # qce_kshard_estimate), so memory does not grow with the number of steps between finish() calls.  The step
        # dropped here is safe for torch's allocator to reuse only on a stream ordered behind that wait: torch's current
        # stream when the step ran on it; otherwise the tensors are recorded on the step's stream, whose
        # work now includes the wait, so the allocator holds them until it has passed.
        keep = (self._keep or []) + [(y, out, int(stream))]
        if len(keep) > 2:
            for yy, oo, s in keep[:-2]:
                if s != cur.cuda_stream:
                    ext = torch.cuda.ExternalStream(s, device=y.device)
                    yy.record_stream(ext)
                    oo.record_stream(ext)
        self._keep = keep[-2:]
        return rows, out

    def finish(self, stream=None):
        """The sync point: flag words read, Cholesky errors raised, flagged rows recombined; `stream` (the caller's)
        is ordered after the steps' collectives."""
        try:
            check(load().qce_kshard_finish(self._h, stream))
        finally:
            self._keep = None

    def flags(self):
        """[rows recombined exactly, Cholesky failure, the same for superseded steps] as the last finish() read them
        (qce_kshard_flags)."""
        out = np.zeros(4)
        check(load().qce_kshard_flags(self._h, ptr(out)))
        return out

    def timing(self, enable):
        check(load().qce_kshard_timing(self._h, int(bool(enable))))

    def kernel_ms(self):
        t, n = ctypes.c_double(), ctypes.c_int()
        check(load().qce_kshard_kernel_ms(self._h, ctypes.byref(t), ctypes.byref(n)))
        return t.value, n.value
