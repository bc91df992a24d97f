"""Outflow preconditioner diagnostics: BiCGStab iterations of one Poisson solve
from a random rhs, and per-step Poisson iterations of the channel from rest, for the line-solve
closure and the wall closure (NSGPU_OUTFLOW_PC) at several channel sizes (square cells)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import navierstokessolver_amd as nsa

sizes = [tuple(int(v) for v in a.split("x")) for a in sys.argv[1:]] or [(1024, 256), (2048, 512), (4096, 1024)]
for nx, ny in sizes:
    h = 4.0 / nx
    for pc in ("line", "wall"):
        os.environ["NSGPU_OUTFLOW_PC"] = pc
        g = nsa.rectangle(nx, ny, lx=4.0, ly=ny * h, bc=[(0, 1.0), (2, 0.0), (4, 0.0), (2, 0.0)])
        s = nsa.GpuSolver(g, h / 8, 1000.0, device=0)
        rng = np.random.default_rng(3)
        s.set(nsa.NS_ARR_PHI, np.zeros(nx * ny))
        s.set(nsa.NS_ARR_RPHI, rng.uniform(-1, 1, nx * ny))
        n, res = s.kernel(nsa.NS_K_POIS_SOLVE)[:2]
        s.close()
        s = nsa.GpuSolver(g, h / 8, 1000.0, device=0)
        its = []
        for _ in range(8):
            try:
                its.append(int(s.step()["it_phi"]))
            except nsa.NsError as e:
                its.append(str(e)[:60])
                break
        s.close()
        print(f"{nx}x{ny} {pc}: random rhs {int(n)} its (res {res:.1e}); steps {its}", flush=True)
