"""SCM multi-path channels on the device: ``SCMMulti`` (reference modules/SCM3GPP/SCMMulti.py:10-63)
backed by ``qce_scm_generate`` (csrc/qce_scm.hip; scm_helper.py:17-84).

``generate_channel(n_batches, n_coherence, n_antennas, rng)`` keeps the reference's signature and
draw order: with a numpy ``Generator`` the path gains, angles and the CN(0,1) spectrum weights are drawn
on the host exactly as the reference draws them (per channel: gains, angles, then crandn(100 N,
n_coherence)), chunk by chunk, and the spectra / partial DFTs run on the device — the reference's
channels to float32 rounding.  ``seed=`` instead draws everything on the device (counter-based, no
host work).  Returns (h (B, n_coherence, N), t (B, N)) complex64 numpy arrays, or device tensors with
``out="device"``.
"""
import numpy as np

from . import _lib


class SCMMulti:
    def __init__(self, path_sigma=2.0, n_path=3, device=0, chunk=512):
        self.path_sigma = path_sigma
        self.n_path = n_path
        self.device = device
        self.chunk = int(chunk)

    def get_config(self):
        return {"path_sigma": self.path_sigma, "n_path": self.n_path}

    def _draws(self, rng, B, n_coherence, N):
        """The reference's per-channel draw sequence (SCMMulti.py:49-53, scm_helper.py:68, utils.py:13-14)."""
        F = 100 * N
        gains = np.empty((B, self.n_path))
        angles = np.empty((B, self.n_path))
        x = np.empty((B, F, n_coherence), dtype=np.complex128)
        for i in range(B):
            g = rng.random(self.n_path)
            gains[i] = g / np.sum(g, axis=0)
            angles[i] = (rng.random(self.n_path) - 0.5) * 180
            x[i] = np.sqrt(0.5) * (rng.standard_normal((F, n_coherence)) + 1j * rng.standard_normal((F, n_coherence)))
        return gains, angles, x

    def generate_channel(self, n_batches, n_coherence, n_antennas, rng=None, *, seed=None, out="host"):
        B, C, N = int(n_batches), int(n_coherence), int(n_antennas)
        lib = _lib.load()
        if out == "device":
            import torch
            dev = torch.device("cuda", self.device)
            h = torch.empty((B, C, N), dtype=torch.complex64, device=dev)
            t = torch.empty((B, N), dtype=torch.complex64, device=dev)
            if rng is not None:
                raise ValueError("out='device' draws on the device: pass seed=, not rng")
            stream = torch.cuda.current_stream(dev).cuda_stream
            _lib.check(lib.qce_scm_generate(B, C, N, self.n_path, float(self.path_sigma), None, None, None,
                                            int(seed or 0), _lib.ptr(h), _lib.ptr(t), self.device, _lib.IO_DEVICE,
                                            stream))
            return h, t
        h = np.empty((B, C, N), dtype=np.complex64)
        t = np.empty((B, N), dtype=np.complex64)
        if rng is None and seed is None:
            rng = np.random.default_rng()
        for s in range(0, B, self.chunk if rng is not None else max(B, 1)):
            e = min(B, s + (self.chunk if rng is not None else B))
            hs, ts = h[s:e], t[s:e]
            if rng is not None:
                g, a, x = self._draws(rng, e - s, C, N)
                _lib.check(lib.qce_scm_generate(e - s, C, N, self.n_path, float(self.path_sigma), _lib.ptr(g),
                                                _lib.ptr(a), _lib.ptr(x), 0, _lib.ptr(hs), _lib.ptr(ts),
                                                self.device, _lib.IO_HOST, None))
            else:
                _lib.check(lib.qce_scm_generate(e - s, C, N, self.n_path, float(self.path_sigma), None, None, None,
                                                int(seed), _lib.ptr(hs), _lib.ptr(ts), self.device, _lib.IO_HOST,
                                                None))
        return h, t
