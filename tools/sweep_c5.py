"""The sweep benchmark (random phi, b from splitmix64 on the device, 10
warm-up + K timed Jacobi sweeps, HIP events): fp64 fields (24 B/cell) and configs[4]'s fp32
fields + fp64 residual (12 B/cell), per grid size.  Under torch.distributed.run each rank
sweeps its x-slab (RCCL ghost rows); the line reports the slowest rank.

  python tools/sweep_c5.py [--n 4096 16384] [--iters 100] [--prec fp64 fp32]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, nargs="+", default=[4096, 16384])
ap.add_argument("--iters", type=int, default=100)
ap.add_argument("--prec", nargs="+", default=["fp64", "fp32"])
a = ap.parse_args()

import torch
import torch.distributed as dist

import navierstokessolver_amd as nsa

rank = int(os.environ.get("RANK", "0"))
world = int(os.environ.get("WORLD_SIZE", "1"))
local = int(os.environ.get("LOCAL_RANK", "0"))
kw = {}
if world > 1:
    from navierstokessolver_amd.dist import nccl_id
    dist.init_process_group("gloo", rank=rank, world_size=world)
    kw = dict(rank=rank, nranks=world, nccl_id=nccl_id(dist))
torch.cuda.set_device(local)
for n in a.n:
    s = nsa.GpuSolver(nsa.cavity(n), 1.0 / (8 * n), 1000.0, poisson=nsa.NS_POISSON_JACOBI, omega=1.0, device=local, **kw)
    for prec in a.prec:
        s.fill_random(0x5EED)
        t = s.time_poisson(10, a.iters) if prec == "fp64" else s.time_poisson_fp32(10, a.iters)
        ms = t["avg_ms"]
        if world > 1:
            x = torch.tensor([ms], dtype=torch.float64)
            dist.all_reduce(x, op=dist.ReduceOp.MAX)
            ms = float(x.item())
        bpc = 24 if prec == "fp64" else 12
        local_cells = (s.i1 - s.i0) * n
        if rank == 0:
            gbs = bpc * local_cells / (ms * 1e-3) / 1e9
            print(json.dumps({"n": n, "prec": prec, "ranks": world, "avg_sweep_us": ms * 1e3,
                              "sweeps_per_s": 1e3 / ms, "glups": n * n / (ms * 1e-3) / 1e9,
                              "per_rank_GBs": gbs, "frac_of_hbm_peak": gbs / 8000.0}), flush=True)
    s.close()
if world > 1:
    dist.destroy_process_group()
