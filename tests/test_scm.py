"""SCM channel generator (SCMMulti.py:30-56, scm_helper.py:17-84).

CPU: the host restatement of the reference's draw order and spectrum (inputs.scm_generate) against the
reference's own generate_channel output in tests/golden/quantizers.npz (make_golden.py).
GPU: scm.SCMMulti through qce_scm_generate — the same golden channels from the same numpy Generator (to
float32 rounding), other shapes against the host restatement, and the on-device draws' statistics
(their own generator: the channel covariance must be toeplitz(t)^T)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN


@pytest.fixture(scope="module")
def kat():
    d = np.load(os.path.join(GOLDEN, "quantizers.npz"), allow_pickle=False)
    return d["scm_h"], d["scm_t"]


def test_host_restatement_matches_reference(kat):
    from quantized_channel_estimation_amd import inputs
    h, t = inputs.scm_generate(4, 1, 16, np.random.default_rng(99), path_sigma=2.0, n_path=3)
    assert np.array_equal(h, kat[0]) and np.array_equal(t, kat[1])


def test_draw_order_matches_host_restatement():
    from quantized_channel_estimation_amd.scm import SCMMulti
    g, a, x = SCMMulti(2.0, 3)._draws(np.random.default_rng(5), 3, 2, 8)
    rng = np.random.default_rng(5)
    for i in range(3):
        gi = rng.random(3)
        assert np.array_equal(g[i], gi / gi.sum())
        assert np.array_equal(a[i], (rng.random(3) - 0.5) * 180)
        xi = np.sqrt(0.5) * (rng.standard_normal((800, 2)) + 1j * rng.standard_normal((800, 2)))
        assert np.array_equal(x[i], xi)


def _close_c64(a, b):
    return np.abs(a - b).max() <= 2e-6 * max(1.0, np.abs(b).max())


@pytest.mark.gpu
def test_gpu_scm_matches_reference(kat):
    from quantized_channel_estimation_amd.scm import SCMMulti
    h, t = SCMMulti(2.0, 3).generate_channel(4, 1, 16, np.random.default_rng(99))
    assert h.dtype == np.complex64 and h.shape == (4, 1, 16) and t.shape == (4, 16)
    assert _close_c64(h, kat[0]) and _close_c64(t, kat[1])


@pytest.mark.gpu
@pytest.mark.parametrize("B,C,N,P", [(5, 3, 64, 3), (3, 1, 100, 1), (2, 2, 200, 5), (7, 1, 32, 2)])
def test_gpu_scm_vs_host_restatement(B, C, N, P):
    from quantized_channel_estimation_amd import inputs
    from quantized_channel_estimation_amd.scm import SCMMulti
    h, t = SCMMulti(2.0, P, chunk=2).generate_channel(B, C, N, np.random.default_rng(B + N))
    ho, to = inputs.scm_generate(B, C, N, np.random.default_rng(B + N), path_sigma=2.0, n_path=P)
    assert _close_c64(h, ho) and _close_c64(t, to)


@pytest.mark.gpu
def test_gpu_scm_device_draws_statistics():
    from scipy.linalg import toeplitz
    from quantized_channel_estimation_amd.scm import SCMMulti
    gen = SCMMulti(2.0, 3)
    h, t = gen.generate_channel(3, 20000, 16, seed=7)
    assert np.allclose(t[:, 0], 1.0, atol=1e-6)  # normalised spectrum: t_0 = sum fs / F = 1
    for b in range(3):
        hb = h[b].astype(np.complex128)  # (n_coherence, N): columns share the channel's spectrum
        Cs = hb.T @ hb.conj() / hb.shape[0]
        Ct = toeplitz(t[b].astype(np.complex128)).T
        assert np.abs(Cs - Ct).max() < 0.06, b
    h2, t2 = gen.generate_channel(3, 20000, 16, seed=7)
    assert np.array_equal(h, h2) and np.array_equal(t, t2)
    h3, _ = gen.generate_channel(3, 10, 16, seed=8)
    assert not np.array_equal(h3, h[:, :10])
    import torch
    hd, td = gen.generate_channel(3, 20000, 16, seed=7, out="device")
    assert torch.equal(hd.cpu(), torch.from_numpy(h)) and torch.equal(td.cpu(), torch.from_numpy(t))
