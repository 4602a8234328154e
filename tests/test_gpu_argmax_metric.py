"""Argmax bit-exactness at the metric configuration (north_star: 'bit-exact for the argmax component index'):
K=128, N=M=64, 'full', 1-bit, 5 dB, the whole metric batch B=10^5 -- where the top-2 gaps of lp shrink toward
1e-5 -- against the FP64 oracle's labels (gmm_cplx_bussgang.py:200-207, :335-349)."""
import numpy as np
import pytest

from conftest import rel_fro

pytestmark = pytest.mark.gpu


def test_argmax_labels_bit_exact_metric_batch():
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import Gmm_nbit, inputs
    K, N, B, snr = 128, 64, 100_000, 5.0
    means, covs, w = inputs.synthetic_model(K, N)
    rng = np.random.default_rng(77)
    hp, _ = inputs.scm_generate(2048, 1, N, rng, n_path=3)
    hp = hp[:, 0, :].astype(complex)
    h = hp[rng.integers(0, hp.shape[0], size=B)]
    y = inputs.get_observation_nbit(h, snr, None, 1, rng=np.random.default_rng(78))
    g = Gmm_nbit.from_params(means, covs, w)
    h1 = g.estimate_from_y(y, snr, N, None, 1, 1)  # mode 1: h = W_j y + b_j, j = argmax lp
    lab = g._predict_cplx(y)  # the observation-domain model of this SNR (the reference's state after the call)
    t = O.prepare(means, covs, np.eye(N), snr, 1)
    gaps = np.empty(B)
    lab_o = np.empty(B, dtype=np.int64)
    for lo in range(0, B, 20_000):
        lp = O.weighted_log_prob(y[lo:lo + 20_000], t["means_y"], t["P"], w)
        lab_o[lo:lo + 20_000] = np.argmax(lp, axis=1)
        s = np.sort(lp, axis=1)
        gaps[lo:lo + 20_000] = s[:, -1] - s[:, -2]
    mism = int((lab != lab_o).sum())
    assert mism == 0, f"{mism} labels differ; min top-2 gap {gaps.min():.3e}"
    # the batch reaches near-ties: the closest top-2 pair is far below the typical gap
    assert gaps.min() < 1e-3, gaps.min()
    # mode 1 picked the same component for every row: its estimate equals the oracle's per-row filter
    sel = np.concatenate([np.arange(0, 2048), np.argsort(gaps)[:512]])
    ho = O.estimate(means, covs, w, y[sel], snr, N, None, 1, 1)
    assert rel_fro(h1[sel], ho) < 1e-9
    print(f"argmax bit-exact over B={B}: min top-2 gap {gaps.min():.3e}, 10 smallest mean {np.sort(gaps)[:10].mean():.3e}")
