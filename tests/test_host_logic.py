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
