"""Generate tests/golden/mofa_fit.npz: golden vectors for the MFA EM (reference
modules/mofa_cplx_bussgang.py:94-115 fit, :219-241 _initialize, :244-265 run_em, :268-320
_EM_per_component / _update_covs, :322-338 _calc_probs, :404-422 _invert_cov_all).

Runs ONLY in the build container (reference imported read-only, no bytecode written, the shims of
make_golden.py plus np.Inf).  For each case: seed numpy's global RNG (the reference's K-means and factor
initialisation draw from it), run the reference's own _initialize on SCM training channels with one BLAS /
OpenMP thread (sklearn's threaded K-means sums centre partials in completion order), snapshot the initial
parameters, run the reference's run_em loop step by step, and store data, the parameters before every
iteration and after the last one (it_*), the final parameters and the lower bound per iteration (L_all).

Usage:  python -B tests/golden/make_golden_mofa_fit.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

CASES = [  # tag, K, latent dim, zero_mean, PPCA, lock_psis, maxiter, seed
    ("zm", 4, 3, True, False, False, 12, 0),
    ("mean", 3, 2, False, False, False, 10, 1),
    ("ppca_lock", 3, 2, False, True, True, 8, 2),
]


def main():
    import warnings
    import numpy as np
    from threadpoolctl import threadpool_limits
    from make_golden import _import_reference
    R = _import_reference()
    np.Inf = np.inf  # mofa_cplx_bussgang.py:302 (numpy 2 removed the alias)
    from modules.mofa_cplx_bussgang import Mofa
    warnings.simplefilter("ignore")
    scm = R["SCMMulti"](path_sigma=2.0, n_path=2)
    h, _ = scm.generate_channel(1200, 1, 16, np.random.default_rng(77))
    data = np.squeeze(h).astype(complex)
    out = dict(data=data)
    tags = []
    for tag, K, M, zm, ppca, lock, maxiter, seed in CASES:
        m = Mofa(n_components=K, latent_dim=M, PPCA=ppca, lock_psis=lock, maxiter=maxiter, tol=1e-14,
                 verbose=False)
        # the state fit() sets before _initialize (:95-100)
        m.zero_mean = zm
        m.N, m.D = data.shape
        m.rs = np.zeros((K, m.N))
        m._covs = np.zeros((K, m.D, m.D), dtype=complex)
        m._inv_covs = np.zeros_like(m._covs)
        np.random.seed(seed)
        with threadpool_limits(limits=1):
            m._initialize(data)
            p = tag + "__"
            out[p + "init_means"] = m._means.copy()
            out[p + "init_lambdas"] = m._lambdas.copy()
            out[p + "init_psis"] = m._psis.copy()
            out[p + "init_amps"] = np.asarray(m.amps).copy()
            # run_em (:244-265) step by step, snapshotting the parameters before every _EM_per_component
            # (device parity is checked per step from these states as well as for the whole fit)
            snaps = {n: [] for n in ("means", "lambdas", "psis", "amps")}
            L, L_all = -np.inf, []
            for i in range(maxiter):
                for n, v in (("means", m._means), ("lambdas", m._lambdas), ("psis", m._psis), ("amps", m.amps)):
                    snaps[n].append(np.array(v, copy=True))
                m._EM_per_component(data, m.PPCA)
                newL = m.logLs.sum()
                L_all.append(newL)
                dL = np.abs((newL - L) / newL)
                if i > 5 and dL < m.tol:
                    break
                L = newL
            m.L_all = L_all
            for n, v in (("means", m._means), ("lambdas", m._lambdas), ("psis", m._psis), ("amps", m.amps)):
                snaps[n].append(np.array(v, copy=True))
                out[p + "it_" + n] = np.stack(snaps[n])
        out[p + "means"] = m._means.copy()
        out[p + "lambdas"] = m._lambdas.copy()
        out[p + "psis"] = m._psis.copy()
        out[p + "amps"] = np.asarray(m.amps).copy()
        out[p + "covs"] = m._covs.copy()
        out[p + "L_all"] = np.asarray(m.L_all, dtype=float)
        out[p + "cfg"] = np.array([K, M, int(zm), int(ppca), int(lock), maxiter, seed])
        tags.append(tag)
    out["tags"] = np.array(tags)
    np.savez_compressed(os.path.join(HERE, "mofa_fit.npz"), **out)
    print("wrote mofa_fit.npz:", tags, {t: len(out[t + "__L_all"]) for t in tags})


if __name__ == "__main__":
    main()
