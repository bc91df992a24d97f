"""The Helmholtz solve's initial guess.  CPU only: the oracle's GPU-algorithm steps
from rest to step s, then RB-SOR sweeps of (I - a L_V) q* = RHS_q (FluidSolver.cpp:547-548) from
  G0  u^n                          (rounds 1-5: with the wall bands first)
  G1  u*^{n-1} = u^n + dt grad phi^{n-1}   (the previous step's Helmholtz solution -- K5 leaves it
                                    in the ping-pong plane, so reading it costs nothing)
  G2  2 u*^{n-1} - u*^{n-2}        (linear extrapolation in time: one more plane read)
and the global sweeps each needs to rtol 1e-8 (with and without the 6 band sweeps).
    python tools/helm_guess_study.py [n=1024] [steps=40] [every=10]"""
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import numpy as np  # noqa: E402
from oracle import OGrid, OSolver, set_threads  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
every = int(sys.argv[3]) if len(sys.argv) > 3 else 10
re = float(os.environ.get("RE", "1000"))
set_threads(os.cpu_count() or 1)
dt = 1.0 / (8 * n)
alpha = dt / (2 * re)
c = alpha * n * n
rho = 4 * c / (1 + 4 * c)
om = 2 / (1 + math.sqrt(1 - rho * rho))
g = OGrid.rectangle(n, n)
s = OSolver(g, dt, re, rtol=1e-8)
s.use_gpu_algorithm(om, 1.1)
ust = []   # u*^k, v*^k of the last steps
for k in range(1, steps + 1):
    s.step()
    st = s.get()
    ust.append((st["u"] + dt * st["gx"], st["v"] + dt * st["gy"]))
    ust = ust[-2:]
    if k % every or k < 3:
        continue
    ru, rv, _, _ = g.rhs_velocity(dt, re, st["u"], st["v"], st["gx"], st["gy"], st["cu"], st["cv"])
    bu, bv = np.linalg.norm(ru), np.linalg.norm(rv)

    def rel(u, v):
        return max(np.linalg.norm(ru - g.apply_helmholtz(alpha, u)) / bu,
                   np.linalg.norm(rv - g.apply_helmholtz(alpha, v)) / bv)

    guesses = {"G0 u^n": (st["u"], st["v"]), "G1 u*^{n-1}": ust[-1],
               "G2 2u*^{n-1}-u*^{n-2}": (2 * ust[-1][0] - ust[0][0], 2 * ust[-1][1] - ust[0][1])}
    out = []
    for name, (u0, v0) in guesses.items():
        for band in (False, True):
            u, v = u0.copy(), v0.copy()
            if band:
                u, v = g.helm_band(alpha, u, v, ru, rv, om)
            hist = [rel(u, v)]
            for _ in range(8):
                u, v, _ = g.helm_sweep(alpha, u, v, ru, rv, om)
                hist.append(rel(u, v))
            need = next((q for q, r in enumerate(hist) if r <= 1e-8), None)
            out.append(f"  {name:24s} band={int(band)} sweeps {need}: " + " ".join(f"{r:.1e}" for r in hist[:6]))
    print(f"n={n} step {k + 1}:\n" + "\n".join(out), flush=True)
