"""The direct solve's own relative residual (one standalone solve, rtol 1e-6: no refinement) per grid, for the
row-pair transforms (NSGPU_FPS_REAL=0) or the one-row real-input ones (=1; set in the environment by the caller)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import navierstokessolver_amd as gpu  # noqa: E402

CAV = [(2, 0.0), (2, 1.0), (2, 0.0), (2, 0.0)]
CHAN = [(0, 1.0), (2, 0.0), (4, 0.0), (2, 0.0)]
for nx, ny, bc in ((300, 4096, CAV), (1024, 1024, CAV), (4096, 4096, CAV), (128, 8192, CAV), (33, 16384, CAV), (4096, 1024, CHAN),
                   (512, 1024, CHAN)):
    h = 4.0 / nx if bc is CHAN else 1.0 / nx
    g = gpu.rectangle(nx, ny, lx=nx * h, ly=ny * h, bc=bc)
    s = gpu.GpuSolver(g, h / 8, 1000.0, rtol=1e-6)
    b = np.random.default_rng(3).uniform(-1, 1, nx * ny)
    s.set(gpu.NS_ARR_PHI, np.zeros(nx * ny))
    s.set(gpu.NS_ARR_RPHI, b)
    its, res = s.kernel(gpu.NS_K_POIS_SOLVE)[:2]
    print("real=%s %dx%d %s its %d res %.3e" % (os.environ.get("NSGPU_FPS_REAL", "1"), nx, ny,
                                                   "chan" if bc is CHAN else "cav", its, res), flush=True)
    s.close()
