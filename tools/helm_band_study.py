"""Where the Helmholtz residual of the guess u^n lives, and what relaxing the wall bands first
buys (k_helm_band).  CPU only: the oracle's GPU-algorithm steps to a developed state,
then numpy RB-SOR on the rectangle's Helmholtz operator (checked against og_apply_helmholtz):
global sweeps to rtol 1e-8 from u^n, and after `sweeps` RB-SOR sweeps restricted to the cells
within `w` of a wall.   python tools/helm_band_study.py [n=4096] [steps=10] [u|v]"""
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import numpy as np  # noqa: E402
from oracle import OGrid, OSolver, set_threads  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
comp = sys.argv[3] if len(sys.argv) > 3 else "u"
set_threads(os.cpu_count() or 1)
dt, re = 1.0 / (8 * n), 1000.0
alpha = dt / (2 * re)
c = alpha * n * n
rho = 4 * c / (1 + 4 * c)
om = 2 / (1 + math.sqrt(1 - rho * rho))
g = OGrid.rectangle(n, n)
s = OSolver(g, dt, re, rtol=1e-8)
s.use_gpu_algorithm(om, 1.1, band=None)
for _ in range(steps):
    s.step()
st = s.get()
ru, rv, _, _ = g.rhs_velocity(dt, re, st["u"], st["v"], st["gx"], st["gy"], st["cu"], st["cv"])
U0 = st[comp].reshape(n, n).copy()
B = (ru if comp == "u" else rv).reshape(n, n)
D = np.full((n, n), 1 + 4 * c)
D[0, :] += c; D[-1, :] += c; D[:, 0] += c; D[:, -1] += c


def apply(U):
    o = D * U
    o[1:, :] -= c * U[:-1, :]; o[:-1, :] -= c * U[1:, :]; o[:, 1:] -= c * U[:, :-1]; o[:, :-1] -= c * U[:, 1:]
    return o


x = np.random.default_rng(0).random(n * n)
assert np.max(np.abs(apply(x.reshape(n, n)).ravel() - g.apply_helmholtz(alpha, x))) < 1e-12
I, J = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
red = (I + J) % 2 == 0
bn = np.linalg.norm(B)


def sweep(U, mask=None):
    for col in (red, ~red):
        m = col if mask is None else (col & mask)
        U[m] += om * (B - apply(U))[m] / D[m]


R = B - apply(U0)
E = R ** 2
print(f"{comp}: ||r||^2 within 16 cells of a wall: {E[(I < 16) | (I >= n - 16) | (J < 16) | (J >= n - 16)].sum() / E.sum():.4f}")
for w, k, part in ((0, 0, "-"), (32, 3, "lid"), (32, 3, "all")):
    U = U0.copy()
    if k:
        m = (J >= n - w) if part == "lid" else ((I < w) | (I >= n - w) | (J < w) | (J >= n - w))
        for _ in range(k):
            sweep(U, m)
    hist = [np.linalg.norm(B - apply(U)) / bn]
    for _ in range(8):
        sweep(U)
        hist.append(np.linalg.norm(B - apply(U)) / bn)
    need = next((q for q, r in enumerate(hist) if r <= 1e-8), None)
    print(f"{comp} band {part} w={w} x{k}: global sweeps to 1e-8: {need}  ", " ".join(f"{r:.1e}" for r in hist))
