"""The oracle (oracle/ns_oracle.c) against the reference's known answers and its own
internal consistency.  Pinning: SURVEY.md section 6 / 8(c) known-answer trace."""
import json
import os

import numpy as np
import pytest

from conftest import KNOWN_TRACE_128, printed_equal
from oracle import OGrid, OSolver

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.slow
def test_known_answer_trace_128_cavity():
    """128^2, Re 100, dt 1/1024, 200 steps: every printed monitor line of SURVEY.md section 6."""
    g = OGrid.rectangle(128, 128)
    s = OSolver(g, 1.0 / 1024, 100.0, rtol=1e-10)
    for it in range(1, 201):
        mm, _ = s.step()
        if it in KNOWN_TRACE_128:
            assert all(printed_equal(a, b) for a, b in zip(mm, KNOWN_TRACE_128[it])), (it, mm)


def test_grid_matches_reference_conventions():
    # cavity vertices clockwise: edges left(-1,0), top(0,1), right(1,0), bottom(0,-1) (Grid.cpp:28-72)
    g = OGrid.rectangle(6, 4)
    assert g.N == 24 and g.nx == 6 and g.ny == 4
    assert np.array_equal(g.id, np.arange(24))                 # id = i*ny + j (Grid.cpp:149-162)
    tag = g.tag.reshape(6, 4, 4)
    assert (tag[0, :, 0] == 0).all() and (tag[:, 3, 3] == 1).all()
    assert (tag[5, :, 1] == 2).all() and (tag[:, 0, 2] == 3).all()
    assert (tag[1:-1, 1:-1] == -1).all()
    np.testing.assert_allclose(g.xc.reshape(6, 4)[:, 0], (np.arange(6) + 0.5) / 6)


def test_l_shaped_polygon_has_compact_ids_and_reentrant_tags():
    # L-shape, clockwise from the origin: 6 edges
    v = [(0, 0), (0, 2), (1, 2), (1, 1), (2, 1), (2, 0)]
    bc = [(2, 0.0)] * 6
    g = OGrid(v, [[0, 2, 8, -1]], [[0, 2, 8, -1]], bc)
    assert g.N == 64 - 16
    ids = g.id.reshape(8, 8)
    assert (ids[4:, 4:] == -1).all()
    assert sorted(ids[ids >= 0].tolist()) == list(range(48))


def test_invalid_grids_rejected():
    with pytest.raises(ValueError):   # counter-clockwise vertex list
        OGrid([(0, 0), (1, 0), (1, 1), (0, 1)], [[0, 1, 4, -1]], [[0, 1, 4, -1]], [(2, 0)] * 4)
    with pytest.raises(ValueError):   # unsupported BC (INLET_PARABOLIC)
        OGrid.rectangle(4, 4, bc=[(1, 1.0), (2, 0), (2, 0), (2, 0)])


def _poisson_setup(n=24, seed=0):
    g = OGrid.rectangle(n, n)
    rng = np.random.default_rng(seed)
    b = rng.uniform(-1, 1, g.N)
    return g, b, b.mean()


def test_sweep_residual_is_true_residual_of_input():
    g, b, m = _poisson_setup()
    phi = np.random.default_rng(1).uniform(-1, 1, g.N)
    r = (b - m) - g.apply_poisson(phi)
    _, r2 = g.rbsor_sweep(phi, b, m, 1.5)
    _, r2j = g.jacobi_sweep(phi, b, m, 0.8)
    assert abs(r2 - (r * r).sum()) <= 1e-9 * (r * r).sum()
    assert abs(r2j - (r * r).sum()) <= 1e-9 * (r * r).sum()


def test_rbsor_converges_to_krylov_solution():
    g, b, m = _poisson_setup(32)
    x, _ = g.solve_poisson(b)
    p = np.zeros(g.N)
    om = 2 / (1 + np.sin(np.pi / 32))
    for _ in range(400):
        p, r2 = g.rbsor_sweep(p, b, m, om)
    assert np.sqrt(r2) <= 1e-9 * np.linalg.norm(b - m)
    np.testing.assert_allclose(p - p.mean(), x - x.mean(), atol=1e-9 * np.abs(x).max())


def test_helmholtz_sweep_converges_to_krylov_solution():
    g = OGrid.rectangle(20, 28, xratio=1.04)
    rng = np.random.default_rng(3)
    ru, rv = rng.uniform(-1, 1, g.N), rng.uniform(-1, 1, g.N)
    alpha = 0.01
    xu, _ = g.solve_helmholtz(alpha, ru)
    u, v = np.zeros(g.N), np.zeros(g.N)
    for _ in range(300):
        u, v, r2 = g.helm_sweep(alpha, u, v, ru, rv, 1.0)
    np.testing.assert_allclose(u, xu, atol=1e-10)
    np.testing.assert_allclose(g.apply_helmholtz(alpha, u), ru, atol=1e-9)


def test_operators_annihilate_constants():
    g = OGrid.rectangle(10, 7, xratio=1.1, yratio=0.9)
    assert np.abs(g.apply_poisson(np.full(g.N, 3.0))).max() < 1e-9
    # wall / inlet phi ghost = phi (FluidSolver.cpp:87-88): constant phi has zero gradient
    gx, gy = g.grad_phi(np.full(g.N, 2.0))
    assert np.abs(gx).max() == 0 and np.abs(gy).max() == 0


def test_golden_fixtures_reproduced():
    """Committed oracle fixtures (tests/golden/make_golden.py) -- guards the restatement."""
    idx = json.load(open(os.path.join(GOLD, "index.json")))
    for case in idx["cases"]:
        d = np.load(os.path.join(GOLD, case["file"]))
        g = OGrid.rectangle(case["nx"], case["ny"], bc=case["bc"], xratio=case["xratio"], yratio=case["yratio"])
        s = OSolver(g, case["dt"], case["re"], rtol=1e-13)
        for k in range(case["steps"]):
            mm, _ = s.step()
            np.testing.assert_allclose(mm, d["mm"][k], rtol=0, atol=1e-11)
        st = s.get()
        np.testing.assert_allclose(st["u"], d["u"], rtol=0, atol=1e-11)
        np.testing.assert_allclose(st["v"], d["v"], rtol=0, atol=1e-11)


def test_helm_band_restatement_is_masked_rbsor():
    """og_helm_band (the GPU's k_helm_band restated) = red-black SOR sweeps of the Helmholtz
    operator applied only on the cells within `width` of a wall, every other cell held: checked
    against an independent numpy restatement (uniform cavity; Dirichlet faces add 2/h^2 to the
    diagonal, FluidSolver.cpp:105-145 + :140-141)."""
    nx, ny, w, sweeps = 64, 48, 10, 3
    dt, re, om = 1.0 / 64, 10.0, 1.1
    alpha = dt / (2 * re)
    g = OGrid.rectangle(nx, ny)
    rng = np.random.default_rng(41)
    u, v, ru, rv = (rng.uniform(-1, 1, nx * ny) for _ in range(4))
    uu, vv = g.helm_band(alpha, u, v, ru, rv, om, width=w, sweeps=sweeps)
    cx, cy = alpha * nx * nx, alpha * ny * ny
    D = np.full((nx, ny), 1 + 2 * cx + 2 * cy)
    D[0, :] += cx; D[-1, :] += cx; D[:, 0] += cy; D[:, -1] += cy

    def apply(U):
        o = D * U
        o[1:, :] -= cx * U[:-1, :]; o[:-1, :] -= cx * U[1:, :]
        o[:, 1:] -= cy * U[:, :-1]; o[:, :-1] -= cy * U[:, 1:]
        return o

    I, J = np.meshgrid(np.arange(nx), np.arange(ny), indexing="ij")
    band = (I < w) | (I >= nx - w) | (J < w) | (J >= ny - w)
    red = (I + J) % 2 == 0
    for q, b, ref in ((u, ru, uu), (v, rv, vv)):
        Q, Bq = q.reshape(nx, ny).copy(), b.reshape(nx, ny)
        for _ in range(sweeps):
            for col in (red, ~red):
                m = col & band
                # one colour at a time: every cell of the colour sees only the other colour's values
                Q[m] += om * (Bq - apply(Q))[m] / D[m]
        assert np.max(np.abs(Q.ravel() - ref)) <= 1e-13 * max(1.0, np.max(np.abs(ref)))
        assert np.array_equal(ref.reshape(nx, ny)[~band], q.reshape(nx, ny)[~band])


def test_multigrid_checks_the_cycle_output():
    """og_mg_solve stops on the residual of a V-cycle's OUTPUT (the GPU's FUSE_P + RES pass): the
    returned cycle count is the first whose output meets rtol."""
    n = 64
    g = OGrid.rectangle(n, n)
    rng = np.random.default_rng(43)
    b = rng.uniform(-1, 1, n * n)
    b -= b.mean()
    rtol = 1e-9
    x, cyc = g.mg_solve(b, rtol=rtol)
    rel = lambda y: np.linalg.norm(b - g.apply_poisson(y)) / np.linalg.norm(b)   # noqa: E731
    assert cyc >= 1 and rel(x) <= rtol
    xm, cm = g.mg_solve(b, rtol=1e-30, maxcycles=cyc - 1)
    assert cm == cyc - 1 and (cyc == 1 or rel(xm) > rtol)


@pytest.mark.parametrize("nx,ny", [(40, 64), (33, 16), (24, 32), (20, 48), (16, 60), (12, 70)])
def test_direct_poisson_restatement(nx, ny):
    """og_fps_solve (the GPU's direct Poisson solve restated: DCT-II along y, Thomas along x with mode
    0 pinned, DCT-III) against an independent sparse LU of the reference's matrix (ConstructLHS,
    FluidSolver.cpp:113-131; one unknown pinned to fix the constant): phi modulo its mean to 1e-11
    of max|phi|, relative residual <= 1e-12."""
    import scipy.sparse as sp
    import scipy.sparse.linalg as spl
    og = OGrid.rectangle(nx, ny, lx=nx / ny)
    assert og.fps_ok()
    rng = np.random.default_rng(nx + ny)
    b = rng.uniform(-1, 1, og.N)
    x = og.fps_solve(b)
    bb = b - b.mean()
    r = og.apply_poisson(x) - bb
    assert np.linalg.norm(r) <= 1e-12 * np.linalg.norm(bb)
    cols = [og.apply_poisson(e) for e in np.eye(og.N)]   # the operator column by column
    A = sp.csc_matrix(np.array(cols).T)
    A = A[1:, 1:]   # x_0 = 0: drop its row and column (the system is consistent)
    xs = np.concatenate([[0.0], spl.spsolve(A.tocsc(), bb[1:])])
    d = (x - x.mean()) - (xs - xs.mean())
    assert np.max(np.abs(d)) <= 1e-11 * np.max(np.abs(xs))


@pytest.mark.parametrize("nx,ny,xr", [(40, 64, 1.03), (33, 16, 0.96), (24, 32, 1.1)])
def test_direct_poisson_restatement_x_stretched(nx, ny, xr):
    """(r6) hx stretched (Grid.cpp:87-92), hy uniform: og_fps_solve's per-row Thomas coefficients + the area
    projection of the plain-mean rhs (b_c -= (sum A b / N) / A_c: the reference's MatNullSpaceRemove leaves the
    stretched system inconsistent, FluidSolver.cpp:550) against an independent sparse LU of the reference's
    matrix on that consistent rhs: phi modulo its mean to 1e-11 of max|phi|, relative residual <= 1e-12."""
    import scipy.sparse as sp
    import scipy.sparse.linalg as spl
    og = OGrid.rectangle(nx, ny, lx=nx / ny, xratio=xr)
    assert og.fps_ok()
    hx = np.diff(np.concatenate([[0.0], np.cumsum(_spacing(nx / ny, nx, xr))]))
    A = np.outer(hx, np.full(ny, 1.0 / ny)).ravel()
    rng = np.random.default_rng(nx + ny + 1)
    b = rng.uniform(-1, 1, og.N)
    x = og.fps_solve(b)
    bb = b - b.mean()
    bc = bb - (np.sum(A * bb) / og.N) / A
    assert abs(np.sum(A * bc)) <= 1e-13 * np.sum(np.abs(A * bc))
    r = og.apply_poisson(x) - bc
    assert np.linalg.norm(r) <= 1e-12 * np.linalg.norm(bc)
    cols = [og.apply_poisson(e) for e in np.eye(og.N)]
    M = sp.csc_matrix(np.array(cols).T)[1:, 1:]   # x_0 = 0 (consistent: the dropped row is implied)
    xs = np.concatenate([[0.0], spl.spsolve(M.tocsc(), bc[1:])])
    d = (x - x.mean()) - (xs - xs.mean())
    assert np.max(np.abs(d)) <= 1e-11 * np.max(np.abs(xs))


def _spacing(length, n, ratio):
    """GenerateFaces' geometric spacing (Grid.cpp:87-92)."""
    h = length * (ratio - 1) / (ratio ** n - 1)
    return np.array([h * ratio ** k for k in range(n)])


def test_direct_poisson_applies_only_to_walled_rectangles_with_uniform_hy():
    assert not OGrid.rectangle(64, 44).fps_ok()                     # ny with a prime factor > 7
    assert not OGrid.rectangle(64, 45).fps_ok()                     # ny odd
    assert OGrid.rectangle(64, 48).fps_ok()                         # (r6) 2^4 * 3: the mixed-radix transforms
    assert not OGrid.rectangle(64, 64, yratio=1.01).fps_ok()        # stretched along y
    assert OGrid.rectangle(64, 64, xratio=1.01).fps_ok()            # (r6) stretched along x only
    assert not OGrid.rectangle(64, 64, bc=[(0, 1.0), (2, 0.0), (4, 0.0), (2, 0.0)]).fps_ok()   # outflow
    assert OGrid.rectangle(64, 64, bc=[(0, 1.0), (2, 0.0), (0, 1.0), (2, 0.5)]).fps_ok()       # inlets
