"""Throughput of the non-cavity paths: a channel with a NEUMANN outflow
(BiCGStab + one-V-cycle preconditioner) and a masked backward-facing step (Jacobi-
preconditioned BiCGStab), from rest, W warm-up + K timed steps.  Prints one line per case."""
import sys
import time

import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import navierstokessolver_amd as nsa


def run(name, grid, dt, re, warm=5, steps=10):
    try:
        _run(name, grid, dt, re, warm, steps)
    except nsa.NsError as e:
        print(f"{name}: FAILED {e}", flush=True)


def _run(name, grid, dt, re, warm, steps):
    torch.cuda.synchronize()
    tc = time.perf_counter()
    s = nsa.GpuSolver(grid, dt, re, device=0)
    torch.cuda.synchronize()
    tc = time.perf_counter() - tc   # (ns_create: a masked domain's capacitance matrix is built here)
    for _ in range(warm):
        s.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st = [s.step() for _ in range(steps)]
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    cells = int(grid.mask.sum())
    print(f"{name}: {cells} cells, {el / steps * 1e3:.2f} ms/step, {cells * steps / el / 1e6:.0f} MLUPS, "
          f"poisson its/step {np.mean([x['it_phi'] for x in st]):.1f}, helmholtz its/step "
          f"{np.mean([x['it_u'] for x in st]):.1f}, set-up {tc:.2f} s", flush=True)
    s.close()


if len(sys.argv) > 2 and sys.argv[1] == "--lshape-only":
    # (r6) the L-shaped cavity alone (a kernel trace of its 2 + 3 steps: tools/evidence.sh fallbacks)
    n = int(sys.argv[2])
    hl = 1.0 / n
    lsh = nsa.polygon([(0, 0), (0, 1), (1, 1), (1, 0.5), (0.5, 0.5), (0.5, 0)], np.full(n, hl), np.full(n, hl),
                      [(2, 0.0), (2, 1.0), (2, 0.0), (2, 0.0), (2, 0.0), (2, 0.0)])
    run(f"L-shaped cavity {n}x{n} (mask, walls)", lsh, hl / 8, 1000.0, warm=2, steps=3)
    sys.exit(0)
nx, ny = int(sys.argv[1]) if len(sys.argv) > 1 else 4096, int(sys.argv[2]) if len(sys.argv) > 2 else 1024
h = 4.0 / nx
run(f"channel {nx}x{ny} (inlet W, outflow E)",
    nsa.rectangle(nx, ny, lx=4.0, ly=ny * h, bc=[(0, 1.0), (2, 0.0), (4, 0.0), (2, 0.0)]), h / 8, 1000.0)
for n in [int(a) for a in sys.argv[3:]] or [256, 512]:
    hs = 2.0 / n
    step = nsa.polygon([(0, 0.5), (0, 1), (2, 1), (2, 0), (0.5, 0), (0.5, 0.5)], np.full(n, hs), np.full(n // 2, hs),
                       [(0, 1.0), (2, 0.0), (4, 0.0), (2, 0.0), (2, 0.0), (2, 0.0)])
    run(f"backward-facing step {n}x{n // 2} (mask, inlet, outflow)", step, hs / 8, 1000.0, warm=2, steps=3)
    hl = 1.0 / n
    lsh = nsa.polygon([(0, 0), (0, 1), (1, 1), (1, 0.5), (0.5, 0.5), (0.5, 0)], np.full(n, hl), np.full(n, hl),
                      [(2, 0.0), (2, 1.0), (2, 0.0), (2, 0.0), (2, 0.0), (2, 0.0)])
    run(f"L-shaped cavity {n}x{n} (mask, walls)", lsh, hl / 8, 1000.0, warm=2, steps=3)
