"""Generate tests/golden/observe.npz: golden vectors for the observation / quantiser row
(reference utils.py:13-14 crandn, :189-203 quant, :241-251 get_observation_nbit).

Runs ONLY in the build container, where the reference checkout exists at /root/reference
(imported read-only, no bytecode written).  The reference's noise generator is the default
argument of ``crandn`` (utils.py:13), created unseeded at import; this script replaces that default
on the imported function object (harness side, never in a reference file) by a seeded generator,
then draws the same CN(0,1) array again from an identically seeded generator so the fixture can
store the noise w the reference added.  Stored per case: h, A (or none), snr, n_bits, thresholds,
labels, w and the reference's y = get_observation_nbit(h, snr, A, n_bits, thr, labels); plus edge
inputs (exact zeros, values on thresholds, NaN, +-inf) through the reference's ``quant``.

Usage:  python -B tests/golden/make_golden_observe.py
"""
import os
import sys

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    if not os.path.isdir(REF):
        raise SystemExit("make_golden_observe.py: /root/reference is absent; the fixture is committed")
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import numpy as np
    np.infty = np.inf
    from modules import utils, lloyd_max_quantizer, uniform_quantizer  # noqa: F401

    out = {}
    rng = np.random.default_rng(77)
    B, N = 300, 32
    h = (rng.standard_normal((B, N)) + 1j * rng.standard_normal((B, N))) * np.sqrt(0.5)
    # a 2-pilot matrix kron(x, I_N) as utils.get_pilot_matrix builds it ('angle_amp')
    A2 = utils.get_pilot_matrix(N, 2, 1, "angle_amp")
    cases = [
        ("b1_snr5", 5.0, None, 1, "uniform"),
        ("b1_snrm10", -10.0, None, 1, "uniform"),
        ("b2u_snr5", 5.0, None, 2, "uniform"),
        ("b3l_snr5", 5.0, None, 3, "lloyd"),
        ("b4u_snr20", 20.0, None, 4, "uniform"),
        ("inf_snr5", 5.0, None, np.inf, "uniform"),
        ("b1_A2", 5.0, A2, 1, "uniform"),
        ("b2u_A2", 5.0, A2, 2, "uniform"),
    ]
    tags = []
    for i, (tag, snr, A, nb, qtype) in enumerate(cases):
        quantizer = utils.get_quantizer([snr], nb, qtype)[snr] if nb not in (1, np.inf) else (None, None, None)
        seed = 1000 + i
        utils.crandn.__kwdefaults__ = {"rng": np.random.default_rng(seed)}
        y = utils.get_observation_nbit(h, snr, A, nb, quantizer[0], quantizer[1])
        M = N if A is None else A.shape[0]
        w = utils.crandn(B, M, rng=np.random.default_rng(seed))  # the reference's own crandn, same seed -> the same draw
        p = tag + "__"
        out[p + "snr"] = np.float64(snr)
        out[p + "n_bits"] = np.float64(nb)
        out[p + "A"] = np.zeros((0, 0), complex) if A is None else np.asarray(A, complex)
        out[p + "w"] = w
        out[p + "y"] = np.asarray(y)
        if quantizer[0] is not None:
            out[p + "thr"] = np.asarray(quantizer[0], float)
            out[p + "lab"] = np.asarray(quantizer[1], float)
        tags.append(tag)
    out["h"] = h
    out["tags"] = np.array(tags)
    # quant edge cases (utils.py:189-203): zeros, values exactly on thresholds, NaN, +-inf
    thr, lab, _ = utils.get_quantizer([5.0], 2, "uniform")[5.0]
    edge = np.array([0.0, -0.0, thr[0], thr[1], thr[2], np.nextafter(thr[1], -1), np.nan, np.inf, -np.inf, 1e300])
    ev = np.empty((edge.size, edge.size), complex)
    ev.real = edge[:, None]
    ev.imag = edge[None, ::-1]
    ev = ev.reshape(-1)
    out["edge_x"] = ev
    out["edge_thr"] = np.asarray(thr, float)
    out["edge_lab"] = np.asarray(lab, float)
    with np.errstate(invalid="ignore"):
        out["edge_q1"] = utils.quant(ev.copy(), 1)
        out["edge_q2"] = utils.quant(ev.copy(), 2, thr, lab)
    np.savez_compressed(os.path.join(HERE, "observe.npz"), **out)
    print("wrote observe.npz:", tags)


if __name__ == "__main__":
    main()
