#!/usr/bin/env python3
"""Probe: does a world-1 RCCL reduce-scatter / all-reduce with a PreMulSum op copy every element for counts that are
not a multiple of 16 doubles?  (r06: the emulated-world rank step lost the last 10 doubles of a 325130-element
reduce-scatter.)  Prints one JSON line per case: the count, the elements that differ from the input."""
import json
import os
import sys

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29561")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
counts = [int(c) for c in sys.argv[1:]] or [325130, 325120, 325121, 325122, 325126, 1000, 1002, 1006, 1010, 16, 18, 26]
for count in counts:
    for opname in ("sum", "premul", "premul_t"):
        x = torch.arange(1, count + 1, dtype=torch.float64, device="cuda")
        out = torch.zeros(count, dtype=torch.float64, device="cuda")
        if opname == "sum":
            op = dist.ReduceOp.SUM
        elif opname == "premul":
            op = dist._make_nccl_premul_sum(1.0)
        else:
            op = dist._make_nccl_premul_sum(torch.ones(1, dtype=torch.float64, device="cuda"))
        dist.reduce_scatter_tensor(out, x, op=op)
        torch.cuda.synchronize()
        bad = (out != x).nonzero().flatten()
        ar = x.clone()
        dist.all_reduce(ar, op=op)
        torch.cuda.synchronize()
        bad_ar = (ar != x).nonzero().flatten()
        print(json.dumps(dict(count=count, op=opname, rs_bad=int(bad.numel()),
                              rs_first_bad=int(bad[0]) if bad.numel() else None, ar_bad=int(bad_ar.numel()))),
              flush=True)
dist.destroy_process_group()
sys.exit(0)
