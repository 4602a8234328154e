import sys, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
from conftest import load_model, case_args, rel_fro
from oracle import qce_oracle as O
from quantized_channel_estimation_amd import Gmm_nbit
for mname in ["full", "synth64"]:
    fx = load_model(mname)
    g = Gmm_nbit.from_params(fx["means_cplx"], fx["covs_cplx"], fx["weights"])
    for tag in fx["cases"]:
        tag = str(tag)
        y, snr, N, A, n_bits, qtype, quantizer = case_args(fx, tag)
        g.estimate_from_y(y, snr, N, A, "all", n_bits, qtype, quantizer)
        lp = g._estimate_weighted_log_prob(y)
        t = g._dev.tables()
        to = O.prepare(fx["means_cplx"], fx["covs_cplx"], A, snr, n_bits, qtype, quantizer)
        lpo = O.weighted_log_prob(y, to["means_y"], to["P"], fx["weights"])
        # lp recomputed on host from the device P
        lph = O.weighted_log_prob(y, t["means_y"], t["P"], fx["weights"])
        cond = max(np.linalg.cond(c) for c in to["Cr"])
        print(f"{mname:8s} {tag:8s} lp-ref {np.max(np.abs(lp-fx[tag+'__lp'])):.2e} lp-oracle {np.max(np.abs(lp-lpo)):.2e} "
              f"hostP-ref {np.max(np.abs(lph-fx[tag+'__lp'])):.2e} P {rel_fro(t['P'], to['P']):.2e} Cr {rel_fro(t['Cr'], to['Cr']):.2e} "
              f"c {np.max(np.abs(t['cconst'] - (2*np.real(O.log_det_cholesky(to['P'])) + np.log(fx['weights']) - A.shape[0]*np.log(np.pi)))):.2e} cond {cond:.1e}")
