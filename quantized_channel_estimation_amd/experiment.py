"""The estimate-and-evaluate loop of Bussgang_GMM.py (:28-340) on the device, end to end: SCM channels
(scm.SCMMulti, device draws), sample covariance, EM fit (Gmm_nbit.fit), quantised observations per SNR
(observe.get_observation_nbit), global / genie Bussgang-LMMSE (baselines.BLMMSE), the GMM estimator, the
scripts' MSE and the statistical rate bound (rate.py).  Returns the script's (mse_list, rate_list) tables
(rows = SNRs after the transpose of :313-314); writing CSV files is left to the caller.

Like the script, every method sees its own observation draw per SNR (:133, :172, :216, :285): four
independent on-device noise streams (seeds seed + 1 + 4 i + j for SNR i, method j).  The MSE and rate of
a method use its own observation.

Table layout: the LS branch's per-sample matched-filter rate (:186-198, rate.matched_filter_rate) is its own
column "LS_glob_mf" -- the script appends it to the previous method's rate row (rate_list[-2]), which a CSV
consumer reading by position must account for; its statistical bound (:200-211) is "LS_glob_stat".
"""
import copy
import warnings

import numpy as np


def run(n_antennas=64, n_components=64, n_summands_or_proba="all", n_path=1, n_bits=2, cov_type="full",
        quantizer_type="uniform", snrs=(-10, -5, 0, 5, 10, 15, 20), n_train=100_000, n_val=10_000,
        zero_mean=True, blocks=None, seed=0, eval_rate=True, max_iter=100, device=0):
    from . import observe, rate
    from .baselines import BLMMSE, LS
    from .gmm import Gmm_nbit
    from .inputs import get_quantizer
    from .scm import SCMMulti
    gen = SCMMulti(path_sigma=2.0, n_path=n_path, device=device)
    h_all, t_all = gen.generate_channel(n_train + n_val, 1, n_antennas, seed=seed)
    h_all = h_all[:, 0, :].astype(np.complex128)
    h_train, h_val, t_val = h_all[:n_train], h_all[n_train:], t_all[n_train:]
    cov = h_train.T @ h_train.conj() / n_train  # sum of outer products / n_train (:119-123)
    quantizer = get_quantizer(list(snrs), n_bits, quantizer_type)
    rate_ok = eval_rate
    mse = {k: [] for k in ("blmmse_glob", "LS_glob", "blmmse_genie", "blmmse_gmm")}
    rates = {k: [] for k in ("blmmse_glob_rstat", "blmmse_genie_rstat", "perfect_rstat", "gmm_rstat",
                         "LS_glob_mf", "LS_glob_stat")}
    gmm = Gmm_nbit(n_components=n_components, covariance_type=cov_type, max_iter=max_iter, device=device)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        gmm.fit(h_train, blocks=blocks, zero_mean=zero_mean)
    for i, snr in enumerate(snrs):
        thr, lab, _ = quantizer[snr]
        r = [observe.get_observation_nbit(h_val, snr, None, n_bits, thr, lab, seed=seed + 1 + 4 * i + j,
                                          device=device) for j in range(4)]
        est = BLMMSE(snr, device=device)
        res = {"blmmse_glob": est.estimate_global(r[0], cov, None, n_bits, quantizer_type, quantizer[snr]),
               "LS_glob": LS(snr, device=device).estimate_global(r[1], cov, None, n_bits, quantizer_type,
                                                                 quantizer[snr]),
               "blmmse_genie": est.estimate_genie(r[2], t_val, None, n_bits, quantizer_type, quantizer[snr]),
               "blmmse_gmm": copy.deepcopy(gmm).estimate_from_y(r[3], snr, n_antennas, None, n_summands_or_proba,
                                                                 n_bits, quantizer_type, quantizer[snr])}
        for k, v in res.items():
            mse[k].append(observe.mse(v, h_val, device=device))
        if rate_ok:
            g, Cq, _ = rate.bussgang_global(cov, snr, n_bits, quantizer[snr], device=device)
            rates["blmmse_glob_rstat"].append(rate.statistical_rate_bound(res["blmmse_glob"], h_val, g, Cq))
            rates["blmmse_genie_rstat"].append(rate.statistical_rate_bound(res["blmmse_genie"], h_val, g, Cq))
            rates["perfect_rstat"].append(rate.statistical_rate_bound(h_val, h_val, g, Cq))
            rates["gmm_rstat"].append(rate.statistical_rate_bound(res["blmmse_gmm"], h_val, g, Cq, norm_clip=1e-1))
            rates["LS_glob_mf"].append(rate.matched_filter_rate(res["LS_glob"], h_val, g, Cq, device=device))
            rates["LS_glob_stat"].append(rate.statistical_rate_bound(res["LS_glob"], h_val, g, Cq))
        else:
            for k in rates:
                rates[k].append(float("nan"))
    mse_list = [["SNR"] + list(snrs)] + [[k] + v for k, v in mse.items()]
    rate_list = [["SNR"] + list(snrs)] + [[k] + v for k, v in rates.items()]
    return [list(x) for x in zip(*mse_list)], [list(x) for x in zip(*rate_list)]
