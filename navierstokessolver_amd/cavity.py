"""Synthetic inputs: the lid-driven cavity of SURVEY.md section 8(d) and the
reference's two input files (grid file Grid.cpp:234-290, sim file
FluidSolver.cpp:626-669) for a rectangle."""
from __future__ import annotations

import numpy as np

from . import _lib as L
from .solver import Edge, GridSpec


def geometric_spacing(a, b, n, ratio):
    """GenerateFaces' spacing rule (Grid.cpp:87-98): ratio -1 = uniform."""
    if ratio == -1:
        return np.full(n, (b - a) / n)
    h = (b - a) * (ratio - 1) / (ratio ** n - 1)
    return np.array([h * ratio ** k for k in range(n)])


def rectangle(nx, ny, lx=1.0, ly=1.0, bc=None, xratio=-1, yratio=-1) -> GridSpec:
    """Rectangle with clockwise vertices (0,0)->(0,ly)->(lx,ly)->(lx,0), i.e. edges
    left(W), top(N), right(E), bottom(S) in that order (Grid.cpp:28-72).
    bc: 4 (type, info) pairs in that edge order; default = lid-driven cavity."""
    if bc is None:
        bc = [(L.NS_BC_WALL, 0.0), (L.NS_BC_WALL, 1.0), (L.NS_BC_WALL, 0.0), (L.NS_BC_WALL, 0.0)]
    normals = [(-1, 0), (0, 1), (1, 0), (0, -1)]
    edges = [Edge(n[0], n[1], int(t), float(i)) for n, (t, i) in zip(normals, bc)]
    return GridSpec(geometric_spacing(0.0, lx, nx, xratio), geometric_spacing(0.0, ly, ny, yratio), edges)


def cavity(n, lid=1.0) -> GridSpec:
    return rectangle(n, n, bc=[(L.NS_BC_WALL, 0.0), (L.NS_BC_WALL, lid), (L.NS_BC_WALL, 0.0), (L.NS_BC_WALL, 0.0)])


def cavity_dt(n):
    """dt = 1/(8n): lid CFL 0.125, an exact power of two for n = 2^k."""
    return 1.0 / (8 * n)


def grid_file_text(nx, ny, lx=1.0, ly=1.0):
    return (f"Vertices {{\n0 0\n0 {ly}\n{lx} {ly}\n{lx} 0\n}}\n"
            f"Nx {{\n0 {lx} {nx} -1\n}}\nNy {{\n0 {ly} {ny} -1\n}}\n")


def sim_file_text(dt, final_time, re, save_iter, bc):
    lines = "\n".join(f"{t} {i}" for t, i in bc)
    # ends with whitespace after the last value (FluidSolver.cpp:662 quirk)
    return f"BC {{\n{lines}\n}}\ndt {dt!r}\nfinal_time {final_time!r}\nre {re!r}\nsaveIter {save_iter}\n"
