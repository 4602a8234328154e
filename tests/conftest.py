import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
MODELS = ["full", "fullmean", "circ", "bcirc", "synth64"]
MODES = {"all": "all", "top1": 1, "top3": 3, "p09": 0.9}


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def load_model(name):
    return dict(np.load(os.path.join(GOLDEN, f"model_{name}.npz"), allow_pickle=False))


def case_args(fx, tag):
    """(y, snr, N, A, n_bits, qtype, quantizer) for a fixture case, as estimate_from_y takes them."""
    p = tag + "__"
    nb = float(fx[p + "n_bits"])
    n_bits = np.inf if np.isinf(nb) else int(nb)
    qtype = str(fx[p + "qtype"])
    quantizer = (fx[p + "thr"], fx[p + "lab"], None) if (p + "thr") in fx else (None, None, None)
    return fx[p + "y"], float(fx[p + "snr"]), int(fx["N"]), fx[p + "A"], n_bits, qtype, quantizer


def rel_fro(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


@pytest.fixture(scope="session")
def golden_models():
    return {m: load_model(m) for m in MODELS}
