#!/usr/bin/env python3
"""One rank's K-shard step through the library's communicator (qce_kshard_*) at the metric geometry, world 1 over
RCCL by default: prepare (+ the step's shift MAX), chunked partials + reduce-scatters, flag MAX, finish.  Prints one
JSON line (per-step time, summed partial-kernel time, parity of 512 rows against the FP64 oracle and, with
--emulate-world, against the single-GPU estimate of the same rows).

--emulate-world W[:R] (QCE_KSHARD_EMULATE_WORLD) lays the rows out as rank R of a W-GPU step: the shard's K
components over all B rows, but the reduce-scatter and the finalisation of only the rank's B / W rows -- the per-rank
work of the W-GPU step without its wire time.  --K is then the per-rank component count.
Used under rocprofv3 --kernel-trace to show the RCCL kernels next to the estimate kernels (profiles/r0*_kshard_*).

The K-shard, its table sets and the communicator are closed explicitly before exit (--no-close leaves them to the
process teardown: the exit-time test of VERDICT r5 #4)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--N", type=int, default=64)
    ap.add_argument("--B", type=int, default=100_000)
    ap.add_argument("--chunks", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--kind", default="rccl", choices=["rccl", "host"])
    ap.add_argument("--single-buffer", action="store_true", help="no spare table set (prepare not overlapped)")
    ap.add_argument("--reserve", type=int, default=-1,
                    help="CUs the shard's grid leaves free (QCE_OPT_RESERVE_CUS; default: the library's K-shard "
                         "default, QCE_KSHARD_RESERVE_CUS or 0)")
    ap.add_argument("--emulate-world", default="", help="W[:R]: rehearse rank R of a W-GPU step on this world-1 rank")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-close", action="store_true", help="exit without closing the K-shard / communicator")
    a = ap.parse_args()
    if a.emulate_world:
        os.environ["QCE_KSHARD_EMULATE_WORLD"] = a.emulate_world
    import torch
    from quantized_channel_estimation_amd import _lib, inputs
    from quantized_channel_estimation_amd.sharding import ComponentShardEstimator, make_comm
    means, covs, w = inputs.synthetic_model(a.K, a.N)
    rng = np.random.default_rng(5)
    hp, _ = inputs.scm_generate(2048, 1, a.N, rng, n_path=3)
    h = hp[:, 0, :].astype(complex)[rng.integers(0, 2048, size=a.B)]
    y = np.ascontiguousarray(inputs.get_observation_nbit(h, 5.0, None, 1, rng=rng), dtype=np.complex128)
    torch.cuda.set_device(0)
    if a.kind == "host":
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("gloo", rank=0, world_size=1)
    comm = make_comm(0, 1, 0, kind=a.kind)
    est = ComponentShardEstimator(means, covs, w, 0, 1, device=0, comm=comm, double_buffer=not a.single_buffer)
    if a.reserve >= 0:
        est.dev.reserve_cus(a.reserve)
        if getattr(est.native, "spare", None) is not None:
            est.native.spare.reserve_cus(a.reserve)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    yd = torch.from_numpy(y).cuda()
    for _ in range(2):
        est.prepare(None, 5.0, 1)
        est.estimate(yd, chunks=a.chunks, scatter=True, sync=False)
    est.finish()
    torch.cuda.synchronize()
    est.native.timing(True)
    t0 = time.perf_counter()
    hp_ms, he_ms = [], []  # host time of each prepare / estimate call (the calls are asynchronous)
    for _ in range(a.steps):
        c0 = time.perf_counter()
        est.prepare(None, 5.0, 1)
        c1 = time.perf_counter()
        est.estimate(yd, chunks=a.chunks, scatter=True, sync=False)
        c2 = time.perf_counter()
        hp_ms.append((c1 - c0) * 1e3)
        he_ms.append((c2 - c1) * 1e3)
    t_sub = time.perf_counter()
    rows, hk = est.finish()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    kms, nl = est.native.kernel_ms()
    r = rows.cpu().numpy()
    hkn = hk.cpu().numpy()
    rec = dict(kind=a.kind, double_buffer=not a.single_buffer, K=a.K, N=a.N, B=a.B, chunks=a.chunks,
               reserve_cus=a.reserve, emulate_world=a.emulate_world or None, rows=int(r.size), steps=a.steps,
               ms_per_step=dt * 1e3, partial_kernel_ms_per_step=kms / a.steps, launches=nl,
               est_per_s_rank_rows=r.size / dt, host_submit_ms_per_step=(t_sub - t0) * 1e3 / a.steps,
               host_prepare_ms=[round(float(np.median(hp_ms)), 4), round(max(hp_ms), 4)],
               host_estimate_ms=[round(float(np.median(he_ms)), 4), round(max(he_ms), 4)])
    if not a.no_parity:
        from oracle import qce_oracle as O
        ho = O.estimate(means, covs, w, y[r[:512]], 5.0, a.N, None, "all", 1)
        rec["parity_rel_fro"] = float(np.linalg.norm(hkn[:512] - ho) / np.linalg.norm(ho))
        # the same rows through the single-GPU estimate of the same mixture (K-shard vs one GPU)
        dm = _lib.DeviceModel(means, covs, w, device=0)
        dm.prepare(None, 5.0, 1)
        h1 = dm.estimate(yd[torch.from_numpy(r).cuda()]).cpu().numpy()
        rec["vs_single_gpu_rel_fro"] = float(np.linalg.norm(hkn - h1) / np.linalg.norm(h1))
        dm.close()
    print(json.dumps(rec), flush=True)
    if not a.no_close:
        est.close()
        comm.close()


if __name__ == "__main__":
    main()
