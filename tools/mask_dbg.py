"""Debug helper: one masked-domain Poisson solve with the solver's verbose history (tests/polygons.py geometry)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np

import navierstokessolver_amd as nsa
from oracle import OGrid
from polygons import ALL

name = sys.argv[1] if len(sys.argv) > 1 else "lshape_s"
P = ALL[name]
og = OGrid(P["vertices"], P["xspec"], P["yspec"], P["bc"])
gs = nsa.GpuSolver(nsa.polygon(P["vertices"], og.hx, og.hy, P["bc"]), 1.0 / 128, 50.0, rtol=1e-12)
m = gs.grid.mask.ravel()
rng = np.random.default_rng(23)
b = np.zeros(m.size)
b[m] = rng.uniform(-100, 100, og.N)
gs.set(nsa.NS_ARR_PHI, np.zeros(m.size))
gs.set(nsa.NS_ARR_RPHI, b)
try:
    print(gs.kernel(nsa.NS_K_POIS_SOLVE)[:2])
except Exception as e:
    print("ERR", e)
print("rhs after consistency fix: finite", np.isfinite(gs.get(nsa.NS_ARR_RPHI)).all(), "outside max",
      np.abs(gs.get(nsa.NS_ARR_RPHI).ravel()[~m]).max())
