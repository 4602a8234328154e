"""SNR sweep on one GPU with double-buffered per-SNR tables.

The reference's script loop estimates one batch per SNR point (Bussgang_GMM.py:284-287, ``estimate_from_y`` per
point of ``snrs``, :43), each call preceded by its per-SNR precompute (gmm_cplx_bussgang.py:246-328).  The
precompute of point t+1 does not depend on the estimate of point t, so with two table sets (two ``DeviceModel``s
of the same mixture) the prepare of t+1 runs on its own stream beside the estimate of t; it waits only for the
estimate t-1, the last reader of its table set.  On small batches (cfg2: B = 10^4, where the prepare is a quarter
of a serial step) that takes the prepare off the critical path.  Every point's result is the single-model result
at its SNR (the same kernels on the same tables)."""
from . import _lib


class SnrSweep:
    """Two table sets of one mixture on one GPU; ``run`` estimates a list of SNR points, prepares overlapped."""

    def __init__(self, means_cplx, covs_cplx, weights, device=0, precision="f64", reserve_cus=32):
        import torch
        self.models = [_lib.DeviceModel(means_cplx, covs_cplx, weights, device=device) for _ in range(2)]
        for m in self.models:
            if precision != "f64":
                m.set_precision(precision)
            if reserve_cus:  # CUs the estimate's persistent grid leaves to the prepare stream
                m.reserve_cus(reserve_cus)
        self.device = int(device)
        self.N = self.models[0].N
        self.prep_stream = torch.cuda.Stream(torch.device("cuda", self.device))

    def run(self, points, outs=None, stream=None):
        """points: [(A, snr_db, n_bits, quant_kind, thresholds, labels, y)] with y a (B, M) complex128 CUDA tensor;
        returns the list of h tensors (asynchronous on `stream`, default torch's current stream)."""
        import torch
        dev = torch.device("cuda", self.device)
        cs = stream if stream is not None else torch.cuda.current_stream(dev)
        ps = self.prep_stream
        used = [None, None]
        res = []
        ps.wait_stream(cs)  # the points' inputs were produced on the caller's stream
        for t, (A, snr, nb, qk, thr, lab, y) in enumerate(points):
            j = t % 2
            m = self.models[j]
            if used[j] is not None:
                ps.wait_event(used[j])  # estimate t-2 has read this table set
            m.prepare(A, snr, nb, qk, thr, lab, stream=ps.cuda_stream)
            ready = torch.cuda.Event()
            ready.record(ps)
            cs.wait_event(ready)
            out = outs[t] if outs is not None else torch.empty((y.shape[0], self.N), dtype=torch.complex128,
                                                                 device=dev)
            m.estimate(y, _lib.MODE_ALL, 0.0, out=out, stream=cs.cuda_stream)
            done = torch.cuda.Event()
            done.record(cs)
            used[j] = done
            res.append(out)
        return res

    def close(self):
        for m in self.models:
            m.close()
