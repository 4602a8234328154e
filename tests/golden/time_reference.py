"""Timing check of the CPU baseline: the loop-faithful oracle
(oracle.qce_oracle.estimate_loop, timed by bench.py as the reference's CPU path on the GPU box, where the
reference cannot travel) against the reference's own Gmm_nbit.estimate_from_y at cfg1 and cfg2 shapes,
same inputs, one BLAS thread each, best of three.  Runs ONLY in the build container (imports
/root/reference read-only via make_golden's harness) and writes timing_ratio.json (numbers only).

Usage:  python -B tests/golden/time_reference.py
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    from threadpoolctl import threadpool_limits
    from make_golden import _import_reference
    from oracle import qce_oracle as O
    from quantized_channel_estimation_amd import inputs
    R = _import_reference()
    gmm_mod = R["gmm"]
    out = {}
    for name, K, N, B in (("cfg1", 16, 32, 200), ("cfg2", 64, 64, 200)):
        means, covs, w = inputs.synthetic_model(K, N, seed=7)
        rng = np.random.default_rng(11)
        h, _ = inputs.scm_generate(B, 1, N, rng, n_path=3)
        y = inputs.get_observation_nbit(h[:, 0, :].astype(complex), 5.0, None, 1, rng=rng)
        g = gmm_mod.Gmm_nbit(n_components=K, covariance_type="full")
        g.means_cplx, g.covs_cplx, g.gm.weights_ = means, covs, w
        A = np.eye(N, dtype=complex)

        def ref():
            return g.estimate_from_y(y, 5.0, N, A, "all", 1, "uniform", None)

        def port():
            return O.estimate_loop(means, covs, w, y, 5.0, N, None, 1, "uniform", None)

        with threadpool_limits(limits=1):
            hr, hp = ref(), port()
            tr = min(_t(ref) for _ in range(3))
            tp = min(_t(port) for _ in range(3))
        err = float(np.linalg.norm(hp - hr) / np.linalg.norm(hr))
        out[name] = dict(K=K, N=N, B=B, reference_s=tr, estimate_loop_s=tp, ratio=tp / tr, rel_fro=err,
                         reference_est_per_s=B / tr, estimate_loop_est_per_s=B / tp)
        print(name, out[name])
    out["note"] = ("estimate_loop / reference wall-time ratio, 1 BLAS thread, best of 3, prepare included; "
                   "SURVEY.md D4 asks for +-15%")
    json.dump(out, open(os.path.join(HERE, "timing_ratio.json"), "w"), indent=1)
    print("wrote timing_ratio.json")


def _t(fn):
    t0 = time.perf_counter()
    fn()
    return time.perf_counter() - t0


if __name__ == "__main__":
    main()
