"""K1 on a masked domain against the rectangle's (one call of ns_kernel(NS_K_RHS) each, wall-clock over 20 calls
after 3): the 1024^2 L-shape (mask) and the 1024^2 cavity, NSGPU_RHS as set by the caller."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import navierstokessolver_amd as nsa

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
hl = 1.0 / n
lsh = nsa.polygon([(0, 0), (0, 1), (1, 1), (1, 0.5), (0.5, 0.5), (0.5, 0)], np.full(n, hl), np.full(n, hl),
                  [(2, 0.0), (2, 1.0), (2, 0.0), (2, 0.0), (2, 0.0), (2, 0.0)])
for name, grid in (("lshape", lsh), ("cavity", nsa.cavity(n))):
    s = nsa.GpuSolver(grid, hl / 8, 1000.0, device=0)
    m = grid.mask.ravel() if getattr(grid, "mask", None) is not None else None
    rng = np.random.default_rng(5)
    for a in (nsa.NS_ARR_U, nsa.NS_ARR_V, nsa.NS_ARR_PHI):
        x = rng.uniform(-1, 1, n * n)
        if m is not None:
            x[~m] = 0.0
        s.set(a, x)
    for _ in range(3):
        s.kernel(nsa.NS_K_RHS)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        s.kernel(nsa.NS_K_RHS)
    torch.cuda.synchronize()
    print(f"{name} {n}^2 NSGPU_RHS={os.environ.get('NSGPU_RHS', '-')}: {(time.perf_counter() - t0) / 20 * 1e6:.1f} us "
          f"per K1 call (host-timed)", flush=True)
    s.close()
