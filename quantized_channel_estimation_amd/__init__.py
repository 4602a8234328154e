"""MI355X-native Bussgang-GMM channel estimator (drop-in for the estimate path of
benediktfesl/Quantized_Channel_Estimation, modules/gmm_cplx_bussgang.py).

The compute path is libqce.so (hand-written HIP for gfx950, include/qce.h) bound through
ctypes; there is no CPU fallback.
"""
from .gmm import GaussianMixtureCplx, Gmm_nbit, Gmm_quant, mp_gmm  # noqa: F401
from .mofa import Mofa  # noqa: F401
from . import baselines, experiment, inputs, observe, rate, scm  # noqa: F401

__all__ = ["Gmm_nbit", "Gmm_quant", "GaussianMixtureCplx", "mp_gmm", "Mofa", "baselines", "experiment", "inputs", "observe", "rate", "scm"]
