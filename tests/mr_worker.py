"""Worker for tests/test_gpu_multirank.py (launched by torch.distributed.run, 2 ranks).
Runs `steps` cavity steps on an x-slab per rank (both ranks on GPU 0), gathers u, v, phi
on rank 0 and saves them.  --transport host | rccl."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
import torch.distributed as dist

import navierstokessolver_amd as nsa
from navierstokessolver_amd.dist import TorchHostTransport, nccl_id

ap = argparse.ArgumentParser()
ap.add_argument("--xport", default="host")
ap.add_argument("--size", type=int, default=64)
ap.add_argument("--size-y", type=int, default=0)
ap.add_argument("--nsteps", type=int, default=10)
ap.add_argument("--solver", type=int, default=nsa.NS_POISSON_MG)
ap.add_argument("--tol", type=float, default=1e-10)
ap.add_argument("--output", required=True)
ap.add_argument("--bc", default="", help="edge BCs W,N,E,S as type:info,... (default: the cavity)")
ap.add_argument("--ratio", type=float, default=-1.0, help="geometric x and y spacing ratio (Grid.cpp)")
ap.add_argument("--poly", default="", help="a tests/polygons.py geometry instead of the rectangle")
ap.add_argument("--sweep32", type=int, default=0,
                help="instead of time steps: K fp32-field Jacobi sweeps (NS_K_POISSON32) of the random input")
ap.add_argument("--stats-only", action="store_true", help="gather only the per-step stats (large grids)")
ap.add_argument("--hash", action="store_true",
                help="gather each slab's sha256 of u, v, phi (bytes, row-major) instead of the fields (large grids)")
ap.add_argument("--async-steps", action="store_true",
                help="ns_step_async (monitor one call late, realigned here) instead of ns_step")
a = ap.parse_args()
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
n, ny = a.size, a.size_y or a.size
kw = dict(rank=rank, nranks=world, device=0, poisson=a.solver, rtol=a.tol)
if a.xport == "host":
    kw["host_transport"] = TorchHostTransport(dist)
else:
    kw["nccl_id"] = nccl_id(dist)
status = "ok"
try:
    bc = [(int(t), float(i)) for t, i in (e.split(":") for e in a.bc.split(","))] if a.bc else None
    if a.poly:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from oracle import OGrid   # the geometry's spacings (a test helper, not the solve)
        from polygons import ALL
        P = ALL[a.poly]
        og = OGrid(P["vertices"], P["xspec"], P["yspec"], P["bc"])
        n, ny = og.nx, og.ny
        grid = nsa.polygon(P["vertices"], og.hx, og.hy, P["bc"])
    else:
        grid = nsa.rectangle(n, ny, bc=bc, xratio=a.ratio, yratio=a.ratio)
    if a.sweep32:
        kw.update(poisson=nsa.NS_POISSON_JACOBI, omega=0.8)
    gs = nsa.GpuSolver(grid, 1.0 / (8 * n), 100.0, **kw)
    if a.sweep32:
        gs.fill_random(0x5EED)
        mm = [list(gs.kernel(nsa.NS_K_POISSON32, a.sweep32)[:1])]
    elif a.async_steps:
        sts = [gs.step_async() for _ in range(a.nsteps)]
        mm = [list(x.values())[:7] for x in sts]
        last = list(gs.monitor())
        for k in range(a.nsteps):   # step k's monitor arrived with step k + 1 (the last via ns_monitor)
            mm[k][:4] = mm[k + 1][:4] if k + 1 < a.nsteps else last
    else:
        sts = [gs.step() for _ in range(a.nsteps)]
        mm = [list(x.values())[:7] for x in sts]
    # (per step: ghost-row exchange groups and collectives -- r5's collective budget)
    xc = [[x["n_exchanges"], x["n_allreduces"]] for x in sts] if not a.sweep32 else []
    if a.hash:
        import hashlib
        f = gs.fields()
        u, v, phi = (np.frombuffer(hashlib.sha256(np.ascontiguousarray(x).tobytes()).digest(), dtype=np.uint8)[None]
                     for x in f)
    else:
        u, v, phi = (np.zeros((1, ny)),) * 3 if a.stats_only else gs.fields()
except Exception as e:  # report, don't hang the other rank
    status = f"error: {e}"
    u = v = phi = np.zeros((1, ny))
    mm = xc = []
parts = [None] * world
dist.all_gather_object(parts, (status, u, v, phi, mm, xc))
if rank == 0:
    st = [p[0] for p in parts]
    if all(s == "ok" for s in st):
        np.savez(a.output, u=np.concatenate([p[1] for p in parts]), v=np.concatenate([p[2] for p in parts]),
                 phi=np.concatenate([p[3] for p in parts]), mm=np.array(parts[0][4]), xc=np.array(parts[0][5]),
                 status="ok")
    else:
        np.savez(a.output, status="; ".join(st))
dist.barrier()
dist.destroy_process_group()
