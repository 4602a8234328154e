"""Generate tests/golden/bench_configs.npz: the reference's own estimates at every BASELINE.json configuration's
model size (K, N, covariance type, quantiser, SNR), so that parity is pinned to the reference at the benchmark
sizes and not only at the small fitted models of make_golden.py (VERDICT r4 "What's weak" 1).

Runs ONLY in the build container (reference imported read-only through make_golden._import_reference, no bytecode
written).  Per configuration: the bench's synthetic model (`inputs.synthetic_model`, numpy only and seeded; the
fixture keeps a checksum of its tables instead of the 8-34 MB of covariances, and the tests rebuild it), 64 seeded
observations y = Q(h + n) of SCM channels (stored), the quantiser from the reference's own producers (stored), and the
reference's `Gmm_nbit.estimate_from_y` (gmm_cplx_bussgang.py:166-243) in modes 'all' and 1, plus its
`_predict_cplx` labels.  Every configuration also once with non-zero means (0.3 CN(0, 1) per entry, seed 12, as
`bench.py --mean`): the reference's fit default zero_mean=False.

Usage:  python -B tests/golden/make_golden_bench.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

# the BASELINE.json configurations (bench.py CONFIGS) without the batch size
CASES = {
    "metric": dict(K=128, N=64, cov="full", n_bits=1, qtype="uniform", snr=5.0),
    "cfg1": dict(K=16, N=32, cov="full", n_bits=1, qtype="uniform", snr=5.0),
    "cfg2": dict(K=64, N=64, cov="full", n_bits=1, qtype="uniform", snr=5.0),
    "cfg3": dict(K=128, N=64, cov="circulant", n_bits=3, qtype="lloyd", snr=5.0),
    "cfg4": dict(K=256, N=128, cov="full", n_bits=1, qtype="uniform", snr=5.0),
    "cfg5": dict(K=128, N=256, cov="block-circulant", blocks=(4, 64), n_bits=2, qtype="uniform", snr=5.0),
}
B = 64


def model_of(c, mean):
    """The bench model of case c (bench.py make_inputs): returns means, covs, weights."""
    import numpy as np
    from quantized_channel_estimation_amd import inputs
    means, covs, w = inputs.synthetic_model(c["K"], c["N"], cov_type=c["cov"], blocks=c.get("blocks"))
    if mean:
        means = 0.3 * inputs.crandn(c["K"], c["N"], rng=np.random.default_rng(12))
    return means, covs, w


def checksum(means, covs, w):
    """Order-sensitive summary of the model tables (the tests compare it at 1e-12 before using the fixture)."""
    import numpy as np
    k = np.arange(1, covs.size + 1, dtype=float).reshape(covs.shape)
    return np.array([np.sum(covs * k).real, np.sum(covs * k).imag, np.sum(np.abs(covs)),
                     np.sum(means * np.arange(1, means.size + 1).reshape(means.shape)).real,
                     np.sum(np.abs(means)), np.sum(w * np.arange(1, w.size + 1))])


def main():
    import warnings
    import numpy as np
    from make_golden import _import_reference
    from quantized_channel_estimation_amd import inputs
    R = _import_reference()
    ut, gmm_mod = R["ut"], R["gmm"]
    warnings.simplefilter("ignore")
    out = {}
    tags = []
    for ci, (name, c) in enumerate(CASES.items()):
        K, N, snr, nb, qt = c["K"], c["N"], c["snr"], c["n_bits"], c["qtype"]
        if nb == 1:
            quantizer = (None, None, None)
        elif qt == "uniform":
            quantizer = ut.get_quantizer([snr], nb, "uniform")[snr]
        else:
            quantizer = R["lloyd"].load_quantizer(snr, nb)[snr]
        rng = np.random.default_rng(7000 + ci)
        h, _ = inputs.scm_generate(B, 1, N, rng, n_path=3)
        h = h[:, 0, :].astype(np.complex128)
        noise = np.sqrt(0.5) * (rng.standard_normal(h.shape) + 1j * rng.standard_normal(h.shape))
        y = ut.quant(h + 10 ** (-snr / 20) * noise, nb, quantizer[0], quantizer[1])
        for mean in (False, True):
            tag = name + ("_mean" if mean else "")
            means, covs, w = model_of(c, mean)
            g = gmm_mod.Gmm_nbit(n_components=K, covariance_type="full")
            g.means_cplx, g.covs_cplx, g.gm.weights_ = means, covs, w
            p = tag + "__"
            if not mean:  # observations and quantiser are stored once per configuration (under its base tag)
                out[p + "y"] = y
                out[p + "h"] = h
                if quantizer[0] is not None:
                    out[p + "thr"] = np.asarray(quantizer[0], dtype=float)
                    out[p + "lab"] = np.asarray(quantizer[1], dtype=float)
            out[p + "checksum"] = checksum(means, covs, w)
            from copy import deepcopy
            for mtag, mode in (("all", "all"), ("top1", 1)):
                gc = deepcopy(g)
                out[p + "hest_" + mtag] = gc.estimate_from_y(y, snr, N, None, mode, nb, qt, quantizer)
                if mtag == "all":
                    out[p + "labels"] = gc._predict_cplx(y)
            tags.append(tag)
            print(tag, "done", flush=True)
    out["tags"] = np.array(tags)
    np.savez_compressed(os.path.join(HERE, "bench_configs.npz"), **out)
    print("wrote bench_configs.npz:", tags)


if __name__ == "__main__":
    main()
