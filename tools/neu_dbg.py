import os, sys
sys.path.insert(0, "."); sys.path.insert(0, "oracle")
import numpy as np
import navierstokessolver_amd as nsa
rng = np.random.default_rng(11)
nx, ny = 24, 48
bc = [(2, 0.0), (4, 0.0), (2, 0.5), (0, 1.0)]
gs = nsa.GpuSolver(nsa.rectangle(nx, ny, bc=bc), 1.0 / 256, 100.0, rtol=1e-12)
b = 100 * rng.uniform(-1, 1, nx * ny)
gs.set(nsa.NS_ARR_PHI, np.zeros(nx * ny)); gs.set(nsa.NS_ARR_RPHI, b)
try:
    print(gs.kernel(nsa.NS_K_POIS_SOLVE)[:2])
except Exception as e:
    print("ERR", e)
