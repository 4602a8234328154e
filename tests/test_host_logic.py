"""Host-side logic of the package that needs no GPU."""
import numpy as np


def test_digest_cache_only_for_truly_immutable_arrays():
    """a read-only view of a writable base can still change, so the parameter digest is cached only
    for arrays whose whole base chain is read-only and owns its memory; freeze_params() copies such views."""
    from quantized_channel_estimation_amd.gmm import _immutable, Gmm_nbit
    base = np.arange(12.0)
    v = base.view()
    v.flags.writeable = False
    assert not _immutable(v)  # the base is writable
    own = np.arange(12.0)
    own.flags.writeable = False
    assert _immutable(own)
    g = Gmm_nbit(n_components=2, covariance_type="full")
    covs = np.stack([np.eye(3, dtype=complex)] * 2)
    g.means_cplx = np.zeros((2, 3), complex)
    g.covs_cplx = covs[:]  # a view of a writable array
    g.gm.weights_ = np.array([0.5, 0.5])
    g.freeze_params()
    assert _immutable(g.covs_cplx) and _immutable(g.means_cplx) and _immutable(g.gm.weights_)
    covs[0, 0, 0] = 5.0  # the caller's array changes; the frozen copy does not
    assert g.covs_cplx[0, 0, 0] == 1.0


def test_pinned_pool_take_and_give_back_are_thread_safe():
    """blocks returned from other threads while take() searches must never shift the record take() hands
    out -- every block handed out is at least the size asked for, and no record is handed out twice."""
    import threading
    from quantized_channel_estimation_amd import _lib

    class Blk:
        def __init__(self, p, n):
            self.ptr, self.nbytes = p, n

    pool = _lib._PinnedPool(cap_bytes=1 << 62)  # no trimming: the pool never calls into the library here
    sizes = [1000 + 37 * i for i in range(64)]
    for i, n in enumerate(sizes):
        pool.free.append((0x1000 * (i + 1), n))
    seen, errors, lock = [], [], threading.Lock()

    def taker(req):
        for _ in range(200):
            try:
                with pool.lock:
                    have = any(req <= n <= 2 * req for _, n in pool.free)
                if not have:
                    continue
                b = pool.take(req)
                if b.nbytes < req:
                    errors.append((req, b.nbytes))
                with lock:
                    seen.append(b.ptr)
                pool.give_back(b)
            except Exception as e:  # pragma: no cover - surfaced below
                errors.append(repr(e))

    def giver(k):
        for j in range(200):
            pool.give_back(Blk(0x10_0000_0000 + k * 10_000 + j, 1500 + j))

    ths = [threading.Thread(target=taker, args=(r,)) for r in (1000, 1500, 2000, 2500)] + \
        [threading.Thread(target=giver, args=(k,)) for k in range(3)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errors, errors[:5]
    ptrs = [p for p, _ in pool.free]
    assert len(ptrs) == len(set(ptrs))  # every record once


def test_kshard_layout_hook_parsing(monkeypatch):
    """QCE_KSHARD_EMULATE_WORLD="W[:R]" applies to a world-1 communicator only, as in csrc/qce_kshard.hip."""
    from quantized_channel_estimation_amd._lib import kshard_layout
    monkeypatch.delenv("QCE_KSHARD_EMULATE_WORLD", raising=False)
    assert kshard_layout(1, 0) == (1, 0)
    monkeypatch.setenv("QCE_KSHARD_EMULATE_WORLD", "8")
    assert kshard_layout(1, 0) == (8, 0)
    assert kshard_layout(2, 1) == (2, 1)  # a real multi-rank communicator keeps its layout
    monkeypatch.setenv("QCE_KSHARD_EMULATE_WORLD", "8:7")
    assert kshard_layout(1, 0) == (8, 7)
    for bad in ("8:8", "1", "x", "4:-1"):
        monkeypatch.setenv("QCE_KSHARD_EMULATE_WORLD", bad)
        assert kshard_layout(1, 0) == (1, 0), bad
