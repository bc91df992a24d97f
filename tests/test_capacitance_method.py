"""(r5) The masked Poisson solve's capacitance method (ns_solver.cpp cap_setup / cap_solve, ns_fps.hip k_cap_*;
DESIGN.md 4) restated in numpy on the oracle's operators -- CPU, no GPU. The operators are oracle/ns_oracle.c's
og_apply_poisson, the restatement of the reference's assembled matrices (FluidSolver.cpp:105-163) on Grid.cpp:149-185's
polygons and on their bounding boxes. Checked:
  * the identity the method rests on: on the domain's rows, the masked operator is the bounding box's plus one rank-1
    term w_f d_f d_f^T per interface face f = (i in the domain, j outside), d_f = e_i - e_j -- the coupling to the
    cells outside vanishes;
  * the solve as the GPU runs it -- two box solves around the capacitance system, with C's columns and the
    regularisation (+ 1 1^T / m) and border exactly as k_cap_col forms them -- reproduces the masked operator's
    projected-sense solution to 1e-10.  Cases: an L-shape, whose box's walls make the box operator consistent with
    mean-free right-hand sides; a backward-facing step, whose box has the E outflow, so mode 0 is solved in the
    projected sense and the system is bordered by the domain's constant.
The box solve F is the projected-sense solve the GPU's direct solve computes (L x = r + mu 1, mu fixed by
consistency), here by least squares."""
import numpy as np
import pytest

from oracle import OGrid

WALL, NEU = (2, 0.0), (4, 0.0)
CASES = {
    # name: vertices, edge BCs, box BCs (rectangle order W, N, E, S), lx, nx, ny, bordered
    "lshape": ([(0, 0), (0, 1), (1, 1), (1, 0.5), (0.5, 0.5), (0.5, 0)], [WALL, (2, 1.0)] + [WALL] * 4,
               [WALL, (2, 1.0), WALL, WALL], 1.0, 12, 12, False),
    "step": ([(0, 0.5), (0, 1), (2, 1), (2, 0), (0.5, 0), (0.5, 0.5)], [(0, 1.0), WALL, NEU, WALL, WALL, WALL],
             [WALL, WALL, NEU, WALL], 2.0, 16, 8, True),
}


def dense(apply, n):
    A = np.empty((n, n))
    for k in range(n):
        e = np.zeros(n)
        e[k] = 1.0
        A[:, k] = apply(e)
    return A


def projected_solve(L, r):
    """x with L x = r + mu 1 for the mu that makes it consistent (the least-squares solution of [L, -1])."""
    n = L.shape[0]
    sol = np.linalg.lstsq(np.hstack([L, -np.ones((n, 1))]), r, rcond=None)[0]
    return sol[:n]


def setup(name):
    verts, bc, bbc, lx, nx, ny, bordered = CASES[name]
    og = OGrid(verts, [[0, lx, nx, -1]], [[0, 1, ny, -1]], bc)
    ob = OGrid.rectangle(nx, ny, lx=lx, ly=1.0, bc=bbc)
    assert og.nx == nx and og.ny == ny and ob.N == nx * ny
    Ld, Lb = dense(og.apply_poisson, og.N), dense(ob.apply_poisson, ob.N)
    ids = og.id.copy()
    dom = np.flatnonzero(ids >= 0)                 # box index of each domain cell, in compact-id order
    assert np.array_equal(ids[dom], np.arange(og.N))
    hx, hy = lx / nx, 1.0 / ny
    fi, fj, w = [], [], []                         # the interface faces (cap_setup's enumeration)
    for i in range(nx):
        for j in range(ny):
            if ids[i * ny + j] < 0:
                continue
            for di, dj, h in ((-1, 0, hx), (1, 0, hx), (0, -1, hy), (0, 1, hy)):
                a, b = i + di, j + dj
                if 0 <= a < nx and 0 <= b < ny and ids[a * ny + b] < 0:
                    fi.append(i * ny + j)
                    fj.append(a * ny + b)
                    w.append(1.0 / (h * h))
    m = len(fi)
    D = np.zeros((ob.N, m))
    D[fi, np.arange(m)] = 1.0
    D[fj, np.arange(m)] = -1.0
    return og, Ld, Lb, dom, D, np.array(w), bordered


@pytest.mark.parametrize("name", sorted(CASES))
def test_masked_operator_is_box_plus_interface_terms(name):
    og, Ld, Lb, dom, D, w, _ = setup(name)
    Le = Lb + (D * w) @ D.T
    out = np.setdiff1d(np.arange(Lb.shape[0]), dom)
    scale = np.max(np.abs(Ld))
    assert np.max(np.abs(Le[np.ix_(dom, dom)] - Ld)) <= 1e-12 * scale
    assert np.max(np.abs(Le[np.ix_(dom, out)])) <= 1e-12 * scale


@pytest.mark.parametrize("name", sorted(CASES))
def test_capacitance_solve_matches_masked_projected_solve(name):
    og, Ld, Lb, dom, D, w, bordered = setup(name)
    n, m = Lb.shape[0], D.shape[1]
    rng = np.random.default_rng(7)
    b = rng.uniform(-1, 1, og.N)
    qd = b - b.mean()                               # r = b - mean on the domain (k_cap_rhs), 0 outside
    q = np.zeros(n)
    q[dom] = qd
    F = lambda r: projected_solve(Lb, r)            # noqa: E731 (the box's direct solve)
    Dw = D * w
    Z = np.column_stack([F(Dw[:, f]) for f in range(m)])
    C = np.eye(m) + D.T @ Z + 1.0 / m              # k_cap_col
    one_dom = np.zeros(n)
    one_dom[dom] = 1.0
    if bordered:                                    # k_cap_col's border: column -D^T e1, row 1^T
        e1 = F(one_dom)
        M = np.zeros((m + 1, m + 1))
        M[:m, :m] = C
        M[:m, m] = -(D.T @ e1)
        M[m, :m] = 1.0
    else:
        M = C
    Minv = np.linalg.inv(M)                          # (the GPU: Gauss-Jordan without pivoting, k_gj_*)
    z1 = F(q)
    g = D.T @ z1                                     # k_cap_gemv's gather
    y = Minv @ (np.append(g, 0.0) if bordered else g)
    x = F(q - Dw @ y[:m])                            # k_cap_scatter, then the second box solve
    if bordered:
        x = x + y[m] * e1                            # k_cap_axpy's lambda e1
    xd = x[dom]
    ref = projected_solve(Ld, qd)
    p, r = xd - xd.mean(), ref - ref.mean()
    assert np.max(np.abs(p - r)) <= 1e-10 * np.max(np.abs(r))
    res = Ld @ xd - qd
    res -= res.mean()                                # P (L x - q): the masked step's projected residual
    assert np.linalg.norm(res) <= 1e-10 * np.linalg.norm(qd)
