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


TOL = 1e-8   # Grid.h:7


def polygon(vertices, hx, hy, bc) -> GridSpec:
    """An axis-parallel polygon over the cells of spacings hx, hy (starting at its lowest
    x / y), classified as Grid.cpp does: edges and outward normals from consecutive vertices
    (Grid.cpp:28-72), a cell is inside if a ray from its centre towards +x crosses an odd
    number of vertical edges, and a cell face lying on an edge (within TOL, Grid.cpp:292)
    is tagged with that edge -- the last one in vertex order wins (Grid.cpp:131-185).
    bc: (type, info) per edge, in vertex order.  A full rectangle of four edges comes back
    without a mask (the fast path)."""
    V = [(float(x), float(y)) for x, y in vertices]
    if len(bc) != len(V):
        raise ValueError("one (type, info) pair per edge")
    xlo, ylo = min(x for x, _ in V), min(y for _, y in V)
    X = xlo + np.concatenate([[0.0], np.cumsum(hx)])
    Y = ylo + np.concatenate([[0.0], np.cumsum(hy)])
    xc, yc = 0.5 * (X[:-1] + X[1:]), 0.5 * (Y[:-1] + Y[1:])
    nx, ny = len(hx), len(hy)
    cross = np.zeros((nx, ny), dtype=np.int64)
    tag = -np.ones((nx, ny, 4), dtype=np.int32)
    edges = []
    for k, (a, b) in enumerate(zip(V, V[1:] + V[:1])):
        if b[0] == a[0]:
            enx, eny, pos, lo, hi = (-1 if b[1] > a[1] else 1), 0, b[0], min(a[1], b[1]), max(a[1], b[1])
            rows = (yc > lo) & (yc < hi)
            cross += np.outer(pos > xc, rows)
            face = X[:-1] if enx == -1 else X[1:]
            tag[np.outer(np.abs(face - pos) <= TOL, rows), 0 if enx == -1 else 1] = k
        elif b[1] == a[1]:
            enx, eny, pos, lo, hi = 0, (1 if b[0] > a[0] else -1), b[1], min(a[0], b[0]), max(a[0], b[0])
            cols = (xc > lo) & (xc < hi)
            face = Y[:-1] if eny == -1 else Y[1:]
            tag[np.outer(cols, np.abs(face - pos) <= TOL), 2 if eny == -1 else 3] = k
        else:
            raise ValueError("Edges should be parallel to the x-axis or y-axis")
        edges.append(Edge(enx, eny, int(bc[k][0]), float(bc[k][1])))
    inside = cross % 2 == 1
    if inside.all() and len(V) == 4:
        return GridSpec(np.asarray(hx, dtype=np.float64), np.asarray(hy, dtype=np.float64), edges)
    cell_id = np.where(inside, np.cumsum(inside.ravel()).reshape(nx, ny) - 1, -1).astype(np.int32)
    return GridSpec(np.asarray(hx, dtype=np.float64), np.asarray(hy, dtype=np.float64), edges,
                    cell_id.ravel(), tag.ravel())


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
