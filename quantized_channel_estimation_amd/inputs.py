"""Host-side producers of the estimate path's inputs (NumPy/SciPy, seeded).

These mirror the reference's helpers that build what ``estimate_from_y`` consumes — the
3GPP-like SCM channels, pilot matrix, quantiser tables and quantised observations — with an
explicit ``rng`` everywhere (the reference's ``crandn`` default generator is created once at
import and never seeded, utils.py:13).  They are table/input builders, not the estimator:
no part of the estimate path falls back to them.
"""
import numpy as np
from scipy import integrate
from scipy.linalg import toeplitz as _toeplitz
from scipy.stats import norm

# J. Max, "Quantizing for minimum distortion", Table 2 (uniform_quantizer.py:11-12)
MAX_UNIFORM_STEP = {1: 1.596, 2: 0.9957, 3: 0.5860, 4: 0.3352, 5: 0.1881, 6: 0.1041, 7: 0.0569, 8: 0.0308}


def crandn(*shape, rng):
    """Circular complex standard normal (utils.py:13-14)."""
    return np.sqrt(0.5) * (rng.standard_normal(shape) + 1j * rng.standard_normal(shape))


def quant(x, n_bits=1, thresholds=None, quant_labels=None):
    """Per-component quantiser (utils.py:189-203): 1 bit -> (sign Re + j sign Im)/sqrt(2),
    otherwise labels[digitize(.)] on real and imaginary parts."""
    x = np.asarray(x)
    if n_bits == 1:
        return 1 / np.sqrt(2) * (np.sign(np.real(x)) + 1j * np.sign(np.imag(x)))
    lab = np.asarray(quant_labels)
    return lab[np.digitize(np.real(x), thresholds)] + 1j * lab[np.digitize(np.imag(x), thresholds)]


def get_observation_nbit(h, snr, A=None, n_bits=1, thresholds=None, quant_labels=None, rng=None):
    """y = Q(A h + 10^(-snr/20) n), n ~ CN(0, I) (utils.py:241-251); rng is explicit."""
    rng = np.random.default_rng() if rng is None else rng
    h = np.asarray(h)
    y = h.astype(complex) if A is None else (np.asarray(A) @ h.T).T
    y = y + 10 ** (-snr / 20) * crandn(*y.shape, rng=rng)
    if n_bits == "inf" or n_bits == np.inf:
        return y
    return quant(y, n_bits, thresholds, quant_labels)


def get_pilot_matrix(n_antennas, n_pilots, n_bits, pilot_type="angle_amp"):
    """Pilot matrix kron(x, I_N) (utils.py:337-367)."""
    if n_bits == np.inf or n_bits == "inf":
        x = np.ones([n_pilots, 1])
    elif pilot_type == "angle":
        x = np.exp(1j * np.linspace(0, np.pi / 2, num=n_pilots, endpoint=False))[:, None]
    elif pilot_type == "angle_amp":
        x = np.linspace(0.5, 1, num=n_pilots, endpoint=True) * np.exp(
            1j * np.linspace(0, np.pi / 2, num=n_pilots, endpoint=False))
        x = (x * np.sqrt(n_pilots) / np.linalg.norm(x))[:, None]
    elif pilot_type == "ones":
        x = np.ones([n_pilots, 1])
    elif pilot_type == "rand":
        raise NotImplementedError("pilot_type 'rand' draws from the unseeded global RNG in the reference")
    else:
        raise NotImplementedError(f"Pilot type {pilot_type} is not implemented!")
    return np.kron(x, np.eye(n_antennas))


def uniform_step(snr_db, n_bits):
    """uniform_quantizer.py:44-45 (with the asymptotic step above 8 bits, :13-21)."""
    base = MAX_UNIFORM_STEP[n_bits] if n_bits <= 8 else 4 * np.sqrt(n_bits) * 2.0 ** (-n_bits)
    return np.sqrt((1 + 10 ** (-snr_db / 10)) / 2) * base


def uniform_quantizer(snr_db, n_bits):
    """(thresholds (2^b-1,), labels (2^b,), None) of the uniform quantiser (utils.py:537-549)."""
    delta = uniform_step(snr_db, n_bits)
    L = 2 ** n_bits
    thr = np.zeros(L - 1)
    half = (L - 2) // 2
    for nb in range(half):
        thr[nb] = -(half - nb) * delta
        thr[-nb - 1] = (half - nb) * delta
    lab = np.zeros(L)
    lab[:L - 1] = thr - delta / 2
    lab[-1] = thr[-1] + delta / 2
    return thr, lab, None


def lloyd_max_quantizer(levels, mean, variance, max_iter=200):
    """Positive half of a Lloyd-Max quantiser for N(mean, variance) by quadrature
    (lloyd_max_quantizer.py:40-90).  Returns (intervals, centroids, distortion)."""
    max_int = np.clip(3 * np.max(variance), 0, 100)
    intervals = np.zeros(levels + 1)
    intervals[:-1] = np.linspace(0.0, max_int, levels)
    intervals[-1] = np.inf
    centroids = np.zeros(levels)
    sd = variance ** 0.5
    for _ in range(max_iter):
        prev = intervals.copy()
        for j in range(levels):
            try:
                num = integrate.quad(lambda x: x * norm.pdf(x, mean, sd), intervals[j], intervals[j + 1])[0]
                den = integrate.quad(lambda x: norm.pdf(x, mean, sd), intervals[j], intervals[j + 1])[0]
                centroids[j] = num / den
            except ZeroDivisionError:
                centroids[j] = (intervals[j] + intervals[j + 1]) / 2
        intervals[1:levels] = (centroids[1:] + centroids[:-1]) / 2.0
        if np.linalg.norm(prev[:-1] - intervals[:-1]) < 1e-5:
            break
    rho = 0.0
    for j in range(levels):
        rho += integrate.quad(lambda x: (x - centroids[j]) ** 2 * norm.pdf(x, mean, sd), intervals[j],
                              intervals[j + 1])[0]
    return intervals, centroids, rho


def load_quantizer(snr, n_bits):
    """Symmetric Lloyd-Max tables for per-component variance (1 + sigma^2)/2
    (lloyd_max_quantizer.py:24-37): {snr: (thresholds (2^b-1,), labels (2^b,), rho)}."""
    sigma2 = 10 ** (-snr / 10)
    thr, lab, rho = lloyd_max_quantizer(int(2 ** n_bits / 2), 0, 0.5 * (1 + sigma2))
    thr = thr[:-1]
    thr = np.concatenate((np.flip(-thr[1:]), thr))
    lab = np.concatenate((np.flip(-lab), lab))
    return {snr: (thr, lab, rho)}


def get_quantizer(snrs, n_bits, quantizer_type="uniform"):
    """{snr: (thresholds, labels, rho)} (utils.py:531-562), computed serially."""
    out = {}
    for snr in snrs:
        if n_bits == "inf" or n_bits == np.inf or n_bits == 1:
            out[snr] = (None, None, None)
        elif quantizer_type == "uniform":
            out[snr] = uniform_quantizer(snr, n_bits)
        elif quantizer_type == "lloyd":
            out[snr] = load_quantizer(snr, n_bits)[snr]
        else:
            raise NotImplementedError(f"Quantizer type {quantizer_type} not implemented!")
    return out


# ---------------------------------------------------------------------------- SCM channels
def _laplace(theta, angles, weights, sigma):
    scale = sigma / np.sqrt(2)
    x = np.outer(theta, np.ones(angles.size)) - angles
    x = (x + 180) % 360 - 180
    return (weights / (2 * scale) * np.exp(-np.abs(x) / scale)).sum(axis=1)


def _spectrum(u, angles, weights, sigma):
    u = (u + np.pi) % (2 * np.pi) - np.pi
    theta = np.degrees(np.arcsin(u / np.pi))
    v = _laplace(theta, angles, weights, sigma) + _laplace(180 - theta, angles, weights, sigma)
    return np.degrees(2 * np.pi * v / np.sqrt(np.pi ** 2 - u ** 2))


def chan_from_spectrum(n_coherence, n_antennas, angles, weights, sigma, rng):
    """One ULA channel from a Laplacian power-angle spectrum (scm_helper.py:39-84):
    returns h (n_coherence, n_antennas) and the first covariance row t (n_antennas,)."""
    n_freq = 100 * n_antennas
    lattice = np.arange(1 / 3, n_freq + 1 / 3) / n_freq * 2 * np.pi - np.pi
    fs = _spectrum(lattice, angles, weights, sigma).reshape(-1, 1)
    cap = max(1, n_freq)
    fs[np.abs(fs) > cap] = cap
    if np.sum(fs) > 0:
        fs = fs / np.sum(fs) * n_freq
    x = crandn(n_freq, n_coherence, rng=rng)
    h = np.fft.ifft(np.sqrt(fs) * x, axis=0) * np.sqrt(n_freq)
    t = (np.fft.fft(fs, axis=0) / n_freq)[:n_antennas].reshape(n_antennas)
    return h[:n_antennas, :].T, t


def scm_generate(n_batches, n_coherence, n_antennas, rng, path_sigma=2.0, n_path=3):
    """SCMMulti.generate_channel (SCMMulti.py:30-56): h (B, n_coherence, N) c64, t (B, N) c64."""
    h = np.zeros([n_batches, n_coherence, n_antennas], dtype=np.complex64)
    t = np.zeros([n_batches, n_antennas], dtype=np.complex64)
    for i in range(n_batches):
        gains = rng.random(n_path)
        gains = gains / np.sum(gains, axis=0)
        angles = (rng.random(n_path) - 0.5) * 180
        h[i], t[i] = chan_from_spectrum(n_coherence, n_antennas, angles, gains, path_sigma, rng)
    return h, t


def toeplitz_cov(t):
    """Hermitian Toeplitz covariance with first row t: toeplitz(t).T as blmmse.py:28 builds it."""
    t = np.asarray(t, dtype=complex)
    return _toeplitz(t).T


def synthetic_model(K, N, cov_type="full", seed=42, blocks=None):
    """The benchmark model recipe of SURVEY.md §8(d) D2: zero means, Dirichlet(1_K) weights
    (seed 11); 'full' covariances toeplitz(t_k)^T + 1e-6 I from SCM first rows (n_path=3, seed);
    'circulant' / 'block-circulant' F^H diag(c_k) F with c_k ~ Exp(1) + 1e-3 normalised to N (seed 43)."""
    w = np.random.default_rng(11).dirichlet(np.ones(K))
    if cov_type == "full":
        _, t = scm_generate(K, 1, N, np.random.default_rng(seed), n_path=3)
        covs = np.stack([toeplitz_cov(t[k]) + 1e-6 * np.eye(N) for k in range(K)])
    elif cov_type in ("circulant", "block-circulant"):
        rng = np.random.default_rng(43)
        c = rng.exponential(1.0, size=(K, N)) + 1e-3
        c = c / c.sum(axis=1, keepdims=True) * N
        if cov_type == "circulant":
            F = np.fft.fft(np.eye(N)) / np.sqrt(N)
        else:
            n1, n2 = blocks
            F = np.kron(np.fft.fft(np.eye(n1)) / np.sqrt(n1), np.fft.fft(np.eye(n2)) / np.sqrt(n2))
        covs = np.stack([F.conj().T @ np.diag(c[k]) @ F for k in range(K)])
    else:
        raise NotImplementedError(cov_type)
    return np.zeros((K, N), complex), covs, w
