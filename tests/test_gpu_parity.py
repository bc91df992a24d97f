"""GPU parity: every kernel of the time step and the full step against the oracle
(oracle/ns_oracle.c, the CPU restatement of /root/reference/SRC/FluidSolver.cpp).

Tolerances (written per test):
  * single kernels (K1, K3, K5, one K2/K4 sweep): max |gpu - oracle| <= 1e-12 * max|oracle|
    (fp64 both sides; differences are FMA contraction / division rounding only);
  * converged solves: <= 1e-7 relative (GPU rtol 1e-11 vs oracle rtol 1e-13);
  * full time steps at the reference's rtol 1e-8: max|du|, max|dv| <= 1e-6 (SURVEY.md 8(c):
    rtol 1e-8 moves u, v by ~8e-8 after 200 steps at 128^2); phi compared modulo its mean.
"""
import numpy as np
import pytest

from conftest import KNOWN_TRACE_128, printed_equal
from oracle import OGrid, OSolver

pytestmark = pytest.mark.gpu

BC_CAVITY = [(2, 0.0), (2, 1.0), (2, 0.0), (2, 0.0)]
BC_FLOW = [(0, 1.0), (2, 0.0), (0, 1.0), (2, 0.5)]   # inlet W, moving wall N, inlet-as-outlet E, moving wall S
BC_CHANNEL = [(0, 1.0), (2, 0.0), (4, 0.0), (2, 0.0)]  # inlet W, walls N / S, NEUMANN outflow E
BC_OUT_N = [(2, 0.0), (4, 0.0), (2, 0.5), (0, 1.0)]    # inflow from S, outflow N, moving wall E
BC_OUT_WS = [(4, 0.0), (0, -0.5), (0, -1.0), (4, 0.0)]  # inflow N / E, outflow W and S (a corner)


def pair(nsa, nx, ny, dt, re, bc=BC_CAVITY, xratio=-1, yratio=-1, **kw):
    og = OGrid.rectangle(nx, ny, bc=bc, xratio=xratio, yratio=yratio)
    gs = nsa.GpuSolver(nsa.rectangle(nx, ny, bc=bc, xratio=xratio, yratio=yratio), dt, re, **kw)
    return og, gs


def rel(a, b):
    return np.max(np.abs(np.asarray(a).ravel() - np.asarray(b).ravel())) / max(np.max(np.abs(b)), 1e-300)


def rand(rng, n, scale=1.0):
    return scale * rng.uniform(-1, 1, n)


GEOMS = [(24, 24, -1, -1, BC_CAVITY), (20, 33, -1, -1, BC_FLOW), (17, 16, 1.07, 0.95, BC_CAVITY),
         (64, 64, -1, -1, BC_FLOW), (100, 130, 1.01, -1, BC_FLOW), (40, 24, -1, -1, BC_CHANNEL),
         (33, 70, 1.03, 0.97, BC_OUT_N), (30, 26, -1, -1, BC_OUT_WS)]


@pytest.mark.parametrize("nx,ny,xr,yr,bc", GEOMS)
def test_k1_rhs_velocity(gpu, nx, ny, xr, yr, bc):
    rng = np.random.default_rng(1)
    dt, re = 1e-3, 250.0
    og, gs = pair(gpu, nx, ny, dt, re, bc, xr, yr)
    N = nx * ny
    u, v, phi, cu, cv = (rand(rng, N) for _ in range(5))
    for a, x in ((gpu.NS_ARR_U, u), (gpu.NS_ARR_V, v), (gpu.NS_ARR_PHI, phi), (gpu.NS_ARR_CU, cu), (gpu.NS_ARR_CV, cv)):
        gs.set(a, x)
    sums = gs.kernel(gpu.NS_K_RHS)
    gx, gy = og.grad_phi(phi)
    ru, rv, cu1, cv1 = og.rhs_velocity(dt, re, u, v, gx, gy, cu, cv)
    assert rel(gs.get(gpu.NS_ARR_RU), ru) <= 1e-12
    assert rel(gs.get(gpu.NS_ARR_RV), rv) <= 1e-12
    assert rel(gs.get(gpu.NS_ARR_CU), cu1) <= 1e-12
    assert rel(gs.get(gpu.NS_ARR_CV), cv1) <= 1e-12
    assert abs(sums[0] - np.sum(ru * ru)) <= 1e-11 * np.sum(ru * ru)


@pytest.mark.parametrize("nx,ny,xr,yr,bc", GEOMS)
def test_k3_divergence(gpu, nx, ny, xr, yr, bc):
    rng = np.random.default_rng(2)
    dt = 1.0 / 512
    og, gs = pair(gpu, nx, ny, dt, 100.0, bc, xr, yr)
    u, v = rand(rng, nx * ny), rand(rng, nx * ny)
    gs.set(gpu.NS_ARR_U, u); gs.set(gpu.NS_ARR_V, v)
    sums = gs.kernel(gpu.NS_K_DIV)
    ref = og.divergence(dt, u, v)
    assert rel(gs.get(gpu.NS_ARR_RPHI), ref) <= 1e-12
    assert abs(sums[0] - ref.sum()) <= 1e-9 * np.abs(ref).sum()
    assert abs(sums[1] - (ref * ref).sum()) <= 1e-11 * (ref * ref).sum()


@pytest.mark.parametrize("nx,ny,xr,yr,bc", GEOMS)
def test_k5_correct(gpu, nx, ny, xr, yr, bc):
    rng = np.random.default_rng(3)
    dt = 1.0 / 256
    og, gs = pair(gpu, nx, ny, dt, 100.0, bc, xr, yr)
    us, vs, phi = (rand(rng, nx * ny) for _ in range(3))
    gs.set(gpu.NS_ARR_U, us); gs.set(gpu.NS_ARR_V, vs); gs.set(gpu.NS_ARR_PHI, phi)
    mm = gs.kernel(gpu.NS_K_CORRECT)
    u, v, _, _ = og.correct(dt, us, vs, phi)
    assert rel(gs.get(gpu.NS_ARR_U), u) <= 1e-12
    assert rel(gs.get(gpu.NS_ARR_V), v) <= 1e-12
    np.testing.assert_allclose(mm[:4], [u.min(), u.max(), v.min(), v.max()], rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize("nx,ny", [(24, 24), (37, 130), (130, 40), (256, 256)])
def test_k4_rbsor_sweeps(gpu, nx, ny):
    """Fused red-black SOR sweeps == the oracle's two-colour sweep (tile seams included)."""
    rng = np.random.default_rng(4)
    og, gs = pair(gpu, nx, ny, 1e-3, 100.0, omega=1.7)
    phi, b = rand(rng, nx * ny), rand(rng, nx * ny, 50.0)
    gs.set(gpu.NS_ARR_PHI, phi); gs.set(gpu.NS_ARR_RPHI, b)
    shift = b.mean()
    p = phi.copy()
    for k in range(3):
        p, r2 = og.rbsor_sweep(p, b, shift, 1.7)
    out = gs.kernel(gpu.NS_K_POISSON, 3)
    assert rel(gs.get(gpu.NS_ARR_PHI), p) <= 1e-12
    assert abs(out[0] - r2) <= 1e-10 * r2        # residual of the last sweep's input


@pytest.mark.parametrize("nx,ny", [(24, 24), (37, 130), (256, 256)])
def test_k4_jacobi_sweeps(gpu, nx, ny):
    rng = np.random.default_rng(5)
    og, gs = pair(gpu, nx, ny, 1e-3, 100.0, poisson=gpu.NS_POISSON_JACOBI, omega=0.8)
    phi, b = rand(rng, nx * ny), rand(rng, nx * ny, 50.0)
    gs.set(gpu.NS_ARR_PHI, phi); gs.set(gpu.NS_ARR_RPHI, b)
    p = phi.copy()
    for k in range(4):
        p, r2 = og.jacobi_sweep(p, b, b.mean(), 0.8)
    out = gs.kernel(gpu.NS_K_POISSON, 4)
    assert rel(gs.get(gpu.NS_ARR_PHI), p) <= 1e-12
    assert abs(out[0] - r2) <= 1e-10 * r2


@pytest.mark.parametrize("nx,ny,xr", [(24, 24, -1), (37, 130, -1), (256, 256, -1), (70, 1000, -1), (40, 5, -1),
                                       (33, 300, 1.02)])
def test_k4_jacobi_fp32_fields(gpu, nx, ny, xr):
    """configs[4]'s fp32-field Jacobi sweep (NS_K_POISSON32): phi, b stored as floats, each
    update and the residual in fp64.  Tolerances: vs the oracle's fp64 sweep with the iterate
    rounded to fp32 after every sweep (the same arithmetic), <= 1e-6 relative (a few fp32 ulps
    where FMA contraction flips a rounding); vs the plain fp64 sweeps <= 1e-5 relative (the
    fp32-field bound; SURVEY.md 8(c) allows 1e-4)."""
    rng = np.random.default_rng(15)
    og, gs = pair(gpu, nx, ny, 1e-3, 100.0, xratio=xr, yratio=xr, poisson=gpu.NS_POISSON_JACOBI, omega=0.8)
    phi, b = rand(rng, nx * ny), rand(rng, nx * ny, 50.0)
    gs.set(gpu.NS_ARR_PHI, phi); gs.set(gpu.NS_ARR_RPHI, b)
    f32 = lambda a: np.asarray(a, dtype=np.float32).astype(np.float64)
    b32, p32, p64 = f32(b), f32(phi), phi.copy()
    for k in range(5):
        p, r2 = og.jacobi_sweep(p32, b32, b.mean(), 0.8)
        p32 = f32(p)
        p64, _ = og.jacobi_sweep(p64, b, b.mean(), 0.8)
    out = gs.kernel(gpu.NS_K_POISSON32, 5)
    got = gs.get(gpu.NS_ARR_PHI)
    assert np.array_equal(got, f32(got))                 # the result is the fp32 iterate
    assert rel(got, p32) <= 1e-6
    assert rel(got, p64) <= 1e-5
    assert abs(out[0] - r2) <= 1e-6 * r2                 # fp64-summed residual of the last input


@pytest.mark.parametrize("nx,ny,xr", [(24, 24, -1), (37, 130, -1), (40, 33, 1.05)])
def test_k2_helmholtz_sweeps(gpu, nx, ny, xr):
    rng = np.random.default_rng(6)
    dt, re = 1.0 / 64, 10.0   # alpha/h^2 ~ O(1): a non-trivial operator
    og, gs = pair(gpu, nx, ny, dt, re, xratio=xr, omega_v=1.0)
    alpha = dt / (2 * re)
    u, v, ru, rv = (rand(rng, nx * ny) for _ in range(4))
    for a, x in ((gpu.NS_ARR_U, u), (gpu.NS_ARR_V, v), (gpu.NS_ARR_RU, ru), (gpu.NS_ARR_RV, rv)):
        gs.set(a, x)
    uu, vv = u.copy(), v.copy()
    for k in range(2):
        uu, vv, r2 = og.helm_sweep(alpha, uu, vv, ru, rv, 1.0)
    out = gs.kernel(gpu.NS_K_HELMHOLTZ, 2)
    assert rel(gs.get(gpu.NS_ARR_U), uu) <= 1e-12
    assert rel(gs.get(gpu.NS_ARR_V), vv) <= 1e-12
    assert abs(out[0] + out[1] - r2) <= 1e-10 * r2


def test_converged_solves(gpu):
    rng = np.random.default_rng(7)
    n, dt, re = 48, 1.0 / 128, 50.0
    og, gs = pair(gpu, n, n, dt, re, rtol=1e-11)
    alpha = dt / (2 * re)
    ru, rv = rand(rng, n * n), rand(rng, n * n)
    gs.set(gpu.NS_ARR_U, np.zeros(n * n)); gs.set(gpu.NS_ARR_V, np.zeros(n * n))
    gs.set(gpu.NS_ARR_RU, ru); gs.set(gpu.NS_ARR_RV, rv)
    its, res = gs.kernel(gpu.NS_K_HELM_SOLVE)[:2]
    assert res <= 1e-11 and its > 0
    xu, _ = og.solve_helmholtz(alpha, ru)
    assert rel(gs.get(gpu.NS_ARR_U), xu) <= 1e-9
    b = rand(rng, n * n, 100.0)
    gs.set(gpu.NS_ARR_PHI, np.zeros(n * n)); gs.set(gpu.NS_ARR_RPHI, b)
    its, res = gs.kernel(gpu.NS_K_POIS_SOLVE)[:2]
    assert res <= 1e-11
    xp, _ = og.solve_poisson(b)
    g = gs.get(gpu.NS_ARR_PHI).ravel()
    assert rel(g - g.mean(), xp - xp.mean()) <= 1e-8


@pytest.mark.parametrize("n,steps,re,bc", [(16, 12, 100.0, BC_CAVITY), (32, 20, 400.0, BC_CAVITY),
                                           (40, 15, 100.0, BC_FLOW)])
def test_full_steps_vs_oracle(gpu, n, steps, re, bc):
    dt = 1.0 / (8 * n)
    og, gs = pair(gpu, n, n, dt, re, bc)
    osv = OSolver(og, dt, re, rtol=1e-13)
    for k in range(steps):
        st = gs.step()
        mm, _ = osv.step()
        np.testing.assert_allclose([st["umin"], st["umax"], st["vmin"], st["vmax"]], mm, atol=1e-6)
    ref = osv.get()
    u, v, phi = gs.fields()
    assert np.max(np.abs(u.ravel() - ref["u"])) <= 1e-6
    assert np.max(np.abs(v.ravel() - ref["v"])) <= 1e-6
    p = phi.ravel() - phi.mean()
    q = ref["phi"] - ref["phi"].mean()
    assert np.linalg.norm(p - q) <= 1e-5 * np.linalg.norm(q)


@pytest.mark.parametrize("nx,ny,bc", [(40, 24, BC_CHANNEL), (64, 64, BC_CHANNEL), (24, 48, BC_OUT_N),
                                      (30, 26, BC_OUT_WS), (33, 20, BC_CHANNEL)])
def test_neumann_outflow_poisson_solve(gpu, nx, ny, bc):
    """NEUMANN outflow: the Poisson matrix gains the 2.5 / -2 / 0.5 ghost rows
    (FluidSolver.cpp:98-101, 147-163); the GPU's BiCGStab (V-cycle preconditioned; a single
    level for the odd 33 x 20) reaches the oracle's BiCGStab solution of the same
    mean-projected system.  Tolerance: 1e-8 relative, phi modulo its mean."""
    rng = np.random.default_rng(11)
    og, gs = pair(gpu, nx, ny, 1.0 / 256, 100.0, bc, rtol=1e-12)
    b = rand(rng, nx * ny, 100.0)
    gs.set(gpu.NS_ARR_PHI, np.zeros(nx * ny)); gs.set(gpu.NS_ARR_RPHI, b)
    its, res = gs.kernel(gpu.NS_K_POIS_SOLVE)[:2]
    assert res <= 1e-12 and 0 < its < 200
    xp, _ = og.solve_poisson(b)   # the oracle solves the outflow system directly
    g = gs.get(gpu.NS_ARR_PHI).ravel()
    err = float(rel(g - g.mean(), xp - xp.mean()))
    assert err <= 1e-8, (err, its)
    with pytest.raises(gpu.NsError):
        gs.kernel(gpu.NS_K_POISSON, 1)   # the smoother's sweeps are not the outflow operator


@pytest.mark.parametrize("nx,ny,steps,re,bc", [(40, 24, 20, 100.0, BC_CHANNEL), (32, 32, 12, 400.0, BC_OUT_N),
                                               (30, 26, 10, 100.0, BC_OUT_WS)])
def test_neumann_outflow_full_steps(gpu, nx, ny, steps, re, bc):
    """Channel-type flows with NEUMANN outflow sides, full steps at the reference's rtol 1e-8
    against the oracle's converged steps: max|du|, max|dv| <= 1e-6 (as for the cavity)."""
    dt = 1.0 / (8 * max(nx, ny))
    og, gs = pair(gpu, nx, ny, dt, re, bc)
    osv = OSolver(og, dt, re, rtol=1e-13)
    for k in range(steps):
        st = gs.step()
        mm, _ = osv.step()
        np.testing.assert_allclose([st["umin"], st["umax"], st["vmin"], st["vmax"]], mm, atol=1e-6)
    ref = osv.get()
    u, v, phi = gs.fields()
    du = float(np.max(np.abs(u.ravel() - ref["u"])))
    dv = float(np.max(np.abs(v.ravel() - ref["v"])))
    assert du <= 1e-6 and dv <= 1e-6, (du, dv)
    p = phi.ravel() - phi.mean()
    q = ref["phi"] - ref["phi"].mean()
    ep = float(np.linalg.norm(p - q) / np.linalg.norm(q))
    assert ep <= 1e-5, ep


@pytest.mark.parametrize("nx,ny,xr,yr,bc", [(32, 32, 1.04, 0.97, BC_CAVITY), (40, 24, 1.02, -1, BC_FLOW),
                                            (48, 32, 0.98, 1.03, BC_CHANNEL), (48, 64, 1.03, -1, BC_CAVITY),
                                            (64, 32, 0.97, -1, BC_FLOW), (64, 64, 1.02, 1.03, BC_CAVITY)])
def test_stretched_full_steps_vs_oracle(gpu, nx, ny, xr, yr, bc):
    """Stretched grids (Grid.cpp ratio > 0): the reference subtracts the PLAIN mean of rhs_phi
    (:550) although the operator's consistency condition is area-weighted, so without an
    outflow side the system it hands the Krylov solver is inconsistent.  The oracle's PCG
    converges to the area-projected solution; the GPU makes the rhs consistent the same way
    (rhs -= m / A_c) and matches it.  With an outflow side both solve P A x = P b.
    Full steps at rtol 1e-8: max|du|, max|dv| <= 1e-6.  (r6) Stretched along x only with ny = 2^p and no outflow:
    the GPU's Poisson solve is the direct one (one 'iteration' per step) on that consistent rhs."""
    dt = 1.0 / (16 * max(nx, ny))
    og, gs = pair(gpu, nx, ny, dt, 200.0, bc, xr, yr)
    osv = OSolver(og, dt, 200.0, rtol=1e-13)
    direct = bc != BC_CHANNEL   # (r6: every walled rectangle -- the FFT or the dense transforms along y)
    for _ in range(10):
        st = gs.step()
        mm, _ = osv.step()
        assert st["it_phi"] < 200, st["it_phi"]
        if direct:
            assert st["it_phi"] == 1, st["it_phi"]
        np.testing.assert_allclose([st["umin"], st["umax"], st["vmin"], st["vmax"]], mm, atol=1e-6)
    ref = osv.get()
    u, v, _ = gs.fields()
    du = float(np.max(np.abs(u.ravel() - ref["u"])))
    dv = float(np.max(np.abs(v.ravel() - ref["v"])))
    assert du <= 1e-6 and dv <= 1e-6, (du, dv)


def test_neumann_needs_multigrid(gpu):
    with pytest.raises(gpu.NsError):
        gpu.GpuSolver(gpu.rectangle(16, 16, bc=BC_CHANNEL), 1e-3, 100.0, poisson=gpu.NS_POISSON_RBSOR)


def test_full_steps_tight_rtol(gpu):
    """At rtol 1e-12 the GPU step converges onto the oracle's discrete solution."""
    n, steps, re = 32, 10, 100.0
    dt = 1.0 / (8 * n)
    og, gs = pair(gpu, n, n, dt, re, rtol=1e-12)
    osv = OSolver(og, dt, re, rtol=1e-13)
    for k in range(steps):
        gs.step()
        osv.step()
    ref = osv.get()
    u, v, _ = gs.fields()
    assert np.max(np.abs(u.ravel() - ref["u"])) <= 1e-9
    assert np.max(np.abs(v.ravel() - ref["v"])) <= 1e-9


def test_known_answer_trace_128(gpu):
    """The reference's printed monitor for the 128^2 Re=100 cavity, at rtol 1e-8."""
    n = 128
    gs = gpu.GpuSolver(gpu.cavity(n), 1.0 / 1024, 100.0)
    for it in range(1, 201):
        st = gs.step()
        if it in KNOWN_TRACE_128:
            got = (st["umin"], st["umax"], st["vmin"], st["vmax"])
            assert all(printed_equal(a, b) for a, b in zip(got, KNOWN_TRACE_128[it])), (it, got)


def test_random_fill_and_timing(gpu):
    n = 512
    gs = gpu.GpuSolver(gpu.cavity(n), 1.0 / (8 * n), 1000.0)
    gs.fill_random(0x5EED)
    phi = gs.get(gpu.NS_ARR_PHI); b = gs.get(gpu.NS_ARR_RPHI)
    assert -1 <= phi.min() < -0.99 and 0.99 < phi.max() < 1
    assert abs(b.mean()) < 0.01
    t = gs.time_poisson(2, 5)
    assert t["avg_ms"] > 0


def test_bad_configs_fail_loudly(gpu):
    with pytest.raises(gpu.NsError):
        gpu.GpuSolver(gpu.rectangle(8, 8, bc=[(1, 1.0), (2, 0.0), (2, 0.0), (2, 0.0)]), 1e-3, 100.0)
    with pytest.raises(gpu.NsError):
        gpu.GpuSolver(gpu.rectangle(8, 8, bc=[(3, 1.0), (2, 0.0), (2, 0.0), (2, 0.0)]), 1e-3, 100.0)
    with pytest.raises(gpu.NsError):
        gpu.GpuSolver(gpu.cavity(8), -1.0, 100.0)


def test_sweeps_deterministic_and_exact_with_many_tiles(gpu):
    """More tiles than can be co-resident (2048^2: 1024 Poisson tiles, 2048 Helmholtz tiles):
    the out-of-place fused sweep is bit-reproducible and equals the oracle's sweep."""
    n = 2048
    runs = []
    for _ in range(2):
        gs = gpu.GpuSolver(gpu.cavity(n), 1.0 / (8 * n), 1000.0, omega=1.99)
        gs.fill_random(7)
        gs.kernel(gpu.NS_K_POISSON, 3)
        runs.append(gs.get(gpu.NS_ARR_PHI))
        if len(runs) == 1:
            phi0 = None
        gs.close()
    assert np.array_equal(runs[0], runs[1])
    gs = gpu.GpuSolver(gpu.cavity(n), 1.0 / (8 * n), 1000.0, omega=1.99)
    gs.fill_random(7)
    phi0 = gs.get(gpu.NS_ARR_PHI).ravel(); b = gs.get(gpu.NS_ARR_RPHI).ravel()
    og = OGrid.rectangle(n, n)
    p = phi0
    for _ in range(3):
        p, _ = og.rbsor_sweep(p, b, b.mean(), 1.99)
    assert rel(runs[0], p) <= 1e-12


@pytest.mark.parametrize("nx,ny", [(64, 64), (96, 160), (100, 60), (33, 47), (256, 512)])
def test_mg_poisson_solve_matches_oracle(gpu, monkeypatch, nx, ny):
    """Multigrid V-cycles converge to the oracle's Krylov solution (odd sizes: RB-SOR fallback).
    (NSGPU_FPS=0: the multigrid also where the direct solve applies, test_gpu_fps.py.)"""
    monkeypatch.setenv("NSGPU_FPS", "0")
    rng = np.random.default_rng(11)
    og, gs = pair(gpu, nx, ny, 1e-3, 100.0, poisson=gpu.NS_POISSON_MG, rtol=1e-11)
    b = rand(rng, nx * ny, 100.0)
    gs.set(gpu.NS_ARR_PHI, np.zeros(nx * ny)); gs.set(gpu.NS_ARR_RPHI, b)
    its, res = gs.kernel(gpu.NS_K_POIS_SOLVE)[:2]
    assert res <= 1e-11
    if nx % 2 == 0 and ny % 2 == 0:
        assert its <= 30, its          # V-cycles, not sweeps
    xp, _ = og.solve_poisson(b)
    g = gs.get(gpu.NS_ARR_PHI).ravel()
    assert rel(g - g.mean(), xp - xp.mean()) <= 1e-8


@pytest.mark.parametrize("direct", [None, "0"])
@pytest.mark.parametrize("nx,ny", [(64, 64), (256, 256), (512, 128), (96, 48), (100, 60)])
def test_mg_vcycles_match_oracle_mg(gpu, monkeypatch, direct, nx, ny):
    """The multigrid solve = the oracle's restatement of the same V(2,2) cycle (og_mg_solve_w, the
    same hierarchy rule) from zero at rtol 1e-10: the same V-cycle count and the same iterate to
    1e-9.  Default (r4): the coarsest level is the first coarse one of <= 128^2 cells, solved exactly
    by its separable eigen-decomposition (k_direct: fp64 MFMA, sides padded to 16 -- 48 x 24 and
    50 x 30 here); NSGPU_DIRECT_CELLS=0: round 3's LDS V-cycle down to <= 16 cells."""
    import oracle as O
    monkeypatch.setenv("NSGPU_FPS", "0")
    if direct is not None:
        monkeypatch.setenv("NSGPU_DIRECT_CELLS", direct)
    O.set_direct_cells(128 * 128 if direct is None else int(direct))
    try:
        rng = np.random.default_rng(23)
        og, gs = pair(gpu, nx, ny, 1e-3, 100.0, poisson=gpu.NS_POISSON_MG, rtol=1e-10)
        b = rand(rng, nx * ny, 100.0)
        gs.set(gpu.NS_ARR_PHI, np.zeros(nx * ny)); gs.set(gpu.NS_ARR_RPHI, b)
        its = gs.kernel(gpu.NS_K_POIS_SOLVE)[0]
        x, cyc = og.mg_solve(b, rtol=1e-10, omega=gs.mg_omega)
        assert its == cyc, (its, cyc)
        g = gs.get(gpu.NS_ARR_PHI).ravel()
        assert rel(g - g.mean(), x - x.mean()) <= 1e-9
    finally:
        O.set_direct_cells(128 * 128)


@pytest.mark.parametrize("solver", ["rbsor", "jacobi_small"])
def test_full_steps_other_poisson_solvers(gpu, solver):
    n, steps, re = 16 if solver == "jacobi_small" else 32, 8, 100.0
    dt = 1.0 / (8 * n)
    kw = dict(poisson=gpu.NS_POISSON_RBSOR) if solver == "rbsor" else dict(poisson=gpu.NS_POISSON_JACOBI, omega=0.9)
    og, gs = pair(gpu, n, n, dt, re, **kw)
    osv = OSolver(og, dt, re, rtol=1e-13)
    for k in range(steps):
        gs.step()
        osv.step()
    ref = osv.get()
    u, v, _ = gs.fields()
    assert np.max(np.abs(u.ravel() - ref["u"])) <= 1e-6
    assert np.max(np.abs(v.ravel() - ref["v"])) <= 1e-6


@pytest.mark.parametrize("nx,ny,xr,yr", [(64, 64, -1, -1), (96, 40, 1.03, -1), (260, 130, -1, 0.99)])
def test_mg_restrict_and_prolong_match_oracle(gpu, nx, ny, xr, yr):
    rng = np.random.default_rng(13)
    og, gs = pair(gpu, nx, ny, 1e-3, 100.0, BC_CAVITY, xr, yr, poisson=gpu.NS_POISSON_MG)
    phi, b = rand(rng, nx * ny), rand(rng, nx * ny, 10.0)
    gs.set(gpu.NS_ARR_PHI, phi); gs.set(gpu.NS_ARR_RPHI, b)
    bc = gs.mg_restrict()
    ref = og.mg_restrict(phi, b, b.mean())
    assert rel(bc, ref) <= 1e-12
    ec = rand(rng, (nx // 2) * (ny // 2))
    gs.mg_prolong(ec)
    assert rel(gs.get(gpu.NS_ARR_PHI), og.mg_prolong(phi, ec)) <= 1e-13


@pytest.mark.parametrize("fps", ["1", "0"])
def test_mg_step_algorithm_matches_oracle_mg(gpu, monkeypatch, fps):
    """Same algorithm on both sides (RB-SOR Helmholtz + the direct Poisson solve, or with
    NSGPU_FPS=0 the multigrid): the CPU baseline leg."""
    monkeypatch.setenv("NSGPU_FPS", fps)
    n, re, steps = 64, 100.0, 8
    dt = 1.0 / (8 * n)
    og, gs = pair(gpu, n, n, dt, re, rtol=1e-10)
    osv = OSolver(og, dt, re, rtol=1e-10)
    osv.use_gpu_algorithm(1.0, fps=fps == "1")
    for _ in range(steps):
        gs.step(); osv.step()
    u, v, _ = gs.fields()
    ref = osv.get()
    assert np.max(np.abs(u.ravel() - ref["u"])) <= 1e-8


@pytest.mark.parametrize("nx,ny,op", [(64, 64, "poisson"), (130, 250, "poisson"), (37, 129, "helmholtz"),
                                      (1024, 512, "poisson"), (700, 300, "helmholtz")])
def test_two_sweep_pass_equals_two_sweeps(gpu, nx, ny, op):
    """The temporally-blocked kernels (two red-black sweeps per HBM pass, k_sweep2; Helmholtz on
    one rank: a three-sweep pass first, k_sweep3) = the oracle's single sweeps, to 1e-12."""
    rng = np.random.default_rng(17)
    if op == "poisson":
        og, gs = pair(gpu, nx, ny, 1e-3, 100.0, omega=1.6)
        phi, b = rand(rng, nx * ny), rand(rng, nx * ny, 30.0)
        gs.set(gpu.NS_ARR_PHI, phi); gs.set(gpu.NS_ARR_RPHI, b)
        p = phi.copy()
        for _ in range(5):
            p, _ = og.rbsor_sweep(p, b, b.mean(), 1.6)
        gs.kernel(gpu.NS_K_POISSON, 5)        # two 2-sweep passes + one single sweep
        assert rel(gs.get(gpu.NS_ARR_PHI), p) <= 1e-12
    else:
        dt, re = 1.0 / 64, 10.0
        og, gs = pair(gpu, nx, ny, dt, re, omega_v=1.1)
        u, v, ru, rv = (rand(rng, nx * ny) for _ in range(4))
        for a, x in ((gpu.NS_ARR_U, u), (gpu.NS_ARR_V, v), (gpu.NS_ARR_RU, ru), (gpu.NS_ARR_RV, rv)):
            gs.set(a, x)
        uu, vv = u.copy(), v.copy()
        for _ in range(5):
            uu, vv, _ = og.helm_sweep(dt / (2 * re), uu, vv, ru, rv, 1.1)
        gs.kernel(gpu.NS_K_HELMHOLTZ, 5)
        assert rel(gs.get(gpu.NS_ARR_U), uu) <= 1e-12
        assert rel(gs.get(gpu.NS_ARR_V), vv) <= 1e-12


@pytest.mark.parametrize("nx,ny,xr,yr,bc", [(64, 64, -1, -1, BC_CAVITY), (300, 517, 1.003, 0.998, BC_FLOW),
                                         (97, 45, -1, -1, BC_FLOW), (520, 390, -1, -1, BC_CAVITY),
                                         (1300, 1100, -1, -1, BC_CAVITY)])
def test_helm_band_matches_oracle(gpu, nx, ny, xr, yr, bc):
    """The Helmholtz wall-band relaxation (k_helm_band: 6 RB-SOR sweeps of u and v on the cells
    within min(nx, ny)/32 >= 32 of a wall, two launches of 32 x 32 tiles with their 6-cell cone in
    LDS) = the oracle's masked sweeps (og_helm_band) to 1e-12; cells off the band keep their
    values bit for bit."""
    rng = np.random.default_rng(31)
    dt, re = 1.0 / 64, 10.0
    og, gs = pair(gpu, nx, ny, dt, re, bc, xr, yr, omega_v=1.1)
    u, v, ru, rv = (rand(rng, nx * ny) for _ in range(4))
    for a, x in ((gpu.NS_ARR_U, u), (gpu.NS_ARR_V, v), (gpu.NS_ARR_RU, ru), (gpu.NS_ARR_RV, rv)):
        gs.set(a, x)
    gs.kernel(gpu.NS_K_HELM_BAND)
    uu, vv = og.helm_band(dt / (2 * re), u, v, ru, rv, 1.1)
    gu, gv = gs.get(gpu.NS_ARR_U).ravel(), gs.get(gpu.NS_ARR_V).ravel()
    assert rel(gu, uu) <= 1e-12
    assert rel(gv, vv) <= 1e-12
    I, J = np.meshgrid(np.arange(nx), np.arange(ny), indexing="ij")
    w = og.band_width()
    far = ((I >= w) & (I < nx - w) & (J >= w) & (J < ny - w)).ravel()
    assert np.array_equal(gu[far], u[far]) and np.array_equal(gv[far], v[far])


def test_helm_band_cuts_sweeps(gpu, monkeypatch):
    """The wall bands first: the same converged steps (rtol 1e-10) in fewer global Helmholtz
    sweeps than from the plain guess u^n (NSGPU_HELM_BAND=0) at the bench's 4096^2 (at 512^2 the
    counts are equal: a smaller a/h^2 converges in fewer sweeps either way)."""
    n, steps = 4096, 3
    out = {}
    for band in ("1", "0"):
        monkeypatch.setenv("NSGPU_HELM_BAND", band)
        gs = gpu.GpuSolver(gpu.cavity(n), 1.0 / (8 * n), 1000.0, rtol=1e-10)
        st = [gs.step() for _ in range(steps)]
        out[band] = (sum(s["it_u"] for s in st), gs.fields())
        gs.close()
    assert out["1"][0] < out["0"][0], (out["1"][0], out["0"][0])
    for a, b in zip(out["1"][1][:2], out["0"][1][:2]):
        assert np.max(np.abs(a - b)) <= 1e-8


@pytest.mark.parametrize("n", [2048, 4096])
def test_two_field_helmholtz_pass_is_bit_identical(gpu, monkeypatch, n):
    """One rank runs a Helmholtz batch of one 3-sweep residual pass per component as ONE
    two-field launch (k_sweep3<FUSE_UV, RES>, strips up to 128 rows); NSGPU_HELM_UV=0 launches u
    and v separately (64-row strips).  Different strips, same arithmetic: the fields, monitors
    and counts of 6 steps are bit-identical, and the two-field batch did run (3-sweep batches)."""
    out = {}
    for uv in ("1", "0"):
        monkeypatch.setenv("NSGPU_HELM_UV", uv)
        gs = gpu.GpuSolver(gpu.cavity(n), 1.0 / (8 * n), 1000.0)
        st = [gs.step() for _ in range(6)]
        out[uv] = (st, gs.fields())
        gs.close()
    (sa, fa), (sb, fb) = out["1"], out["0"]
    assert any(s["it_u"] == 3 for s in sa), [s["it_u"] for s in sa]
    for a, b in zip(sa, sb):
        for k in ("umin", "umax", "vmin", "vmax", "it_u", "it_phi"):
            assert a[k] == b[k], (k, a[k], b[k])
    for x, y in zip(fa, fb):
        assert np.array_equal(x, y), float(np.max(np.abs(x - y)))


@pytest.mark.parametrize("nx,ny", [(256, 192), (96, 160)])
def test_fused_transfer_passes_match_separate_transfers(gpu, monkeypatch, nx, ny):
    """The last pre-smoothing pass with the restriction fused in (k_sweep2 FUSE_R) and the first
    post-smoothing pass with the prolongation fused in (FUSE_P) give the same V-cycles as
    sweeps + k_restrict / k_prolong, and the oracle's solution.  NSGPU_PAIR_MIN_CELLS=0 makes
    every level use the two-sweep passes (production: levels >= 2048^2 only)."""
    rng = np.random.default_rng(23)
    b = rand(rng, nx * ny, 100.0)
    out = {}
    monkeypatch.setenv("NSGPU_FPS", "0")
    monkeypatch.setenv("NSGPU_PAIR_MIN_CELLS", "0")
    for fr, fp in (("1", "1"), ("0", "0"), ("1", "0"), ("0", "1")):
        monkeypatch.setenv("NSGPU_FUSED_RESTRICT", fr)
        monkeypatch.setenv("NSGPU_FUSED_PROLONG", fp)
        og, gs = pair(gpu, nx, ny, 1e-3, 100.0, poisson=gpu.NS_POISSON_MG, rtol=1e-11)
        gs.set(gpu.NS_ARR_PHI, np.zeros(nx * ny)); gs.set(gpu.NS_ARR_RPHI, b)
        its, res = gs.kernel(gpu.NS_K_POIS_SOLVE)[:2]
        out[fr + fp] = (its, res, gs.get(gpu.NS_ARR_PHI).ravel())
        gs.close()
    for k in ("11", "10", "01"):
        assert out[k][0] == out["00"][0], (k, out[k][0], out["00"][0])
        assert out[k][1] <= 1e-11
        assert rel(out[k][2], out["00"][2]) <= 1e-12
    xp, _ = og.solve_poisson(b)
    g = out["11"][2]
    assert rel(g - g.mean(), xp - xp.mean()) <= 1e-8


@pytest.mark.parametrize("nx,ny", [(256, 192), (100, 68), (96, 160)])
def test_tiled_small_level_passes_match_streaming(gpu, monkeypatch, nx, ny):
    """The LDS-tiled fused passes of the small levels (k_tile2: two sweeps + residual +
    restriction; prolongation + two sweeps) give the same V-cycles as the streaming fused
    passes (k_sweep2, NSGPU_PAIR_MIN_CELLS=0) and as single sweeps + separate transfers
    (NSGPU_TILE_SMALL=0): same cycle count, same iterate to 1e-12 (same arithmetic), and the
    oracle's solution.  Partial tiles: 100 x 68."""
    rng = np.random.default_rng(29)
    b = rand(rng, nx * ny, 100.0)
    out = {}
    monkeypatch.setenv("NSGPU_FPS", "0")
    for mode, env in (("tile", {}), ("stream", {"NSGPU_PAIR_MIN_CELLS": "0"}), ("single", {"NSGPU_TILE_SMALL": "0"})):
        for k in ("NSGPU_PAIR_MIN_CELLS", "NSGPU_TILE_SMALL"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        og, gs = pair(gpu, nx, ny, 1e-3, 100.0, poisson=gpu.NS_POISSON_MG, rtol=1e-11)
        gs.set(gpu.NS_ARR_PHI, np.zeros(nx * ny)); gs.set(gpu.NS_ARR_RPHI, b)
        its, res = gs.kernel(gpu.NS_K_POIS_SOLVE)[:2]
        out[mode] = (its, res, gs.get(gpu.NS_ARR_PHI).ravel())
        gs.close()
    for k in ("stream", "single"):
        assert out[k][0] == out["tile"][0], (k, out[k][0], out["tile"][0])
        assert rel(out[k][2], out["tile"][2]) <= 1e-12
    assert out["tile"][1] <= 1e-11
    xp, _ = og.solve_poisson(b)
    g = out["tile"][2]
    assert rel(g - g.mean(), xp - xp.mean()) <= 1e-8


@pytest.mark.parametrize("nx,ny,xr,yr,bc", [(300, 200, 1.002, 0.998, BC_FLOW), (37, 70, -1, -1, BC_CAVITY),
                                            (261, 131, 1.003, -1, BC_CAVITY), (5, 5, -1, -1, BC_CAVITY)])
@pytest.mark.parametrize("mode", ["stream", "stream3", "lds"])
def test_k1_equals_global_kernel(gpu, monkeypatch, mode, nx, ny, xr, yr, bc):
    """K1 as streaming strips (k_rhs_s: each MUSCL slope and face flux once, + the wall ring
    k_rhs_ring; NSGPU_K1S=3 its 3-waves build), or staged in LDS (NSGPU_RHS=lds: k_rhs_lds + the
    wall-cell kernel k_rhs_bc) = the global-load K1 (NSGPU_RHS=global, rhs_cell per cell): the same
    face states and fluxes; the compiler's FMA contraction differs between the kernels, so equal
    to 1e-14 relative (of the field's max), not bit for bit.  Odd ny (the ring's third column),
    a stretched grid, and a grid with no inner cell (5 x 5: all ring) included."""
    rng = np.random.default_rng(31)
    dt, re = 1e-3, 250.0
    N = nx * ny
    ins = [rand(rng, N) for _ in range(5)]
    outs = []
    for mode in (mode, "global"):
        monkeypatch.delenv("NSGPU_RHS", raising=False)
        monkeypatch.delenv("NSGPU_K1S", raising=False)
        if mode == "stream3":
            monkeypatch.setenv("NSGPU_K1S", "3")
        if mode in ("lds", "global"):
            monkeypatch.setenv("NSGPU_RHS", mode)
        _, gs = pair(gpu, nx, ny, dt, re, bc, xr, yr)
        for a, x in zip((gpu.NS_ARR_U, gpu.NS_ARR_V, gpu.NS_ARR_PHI, gpu.NS_ARR_CU, gpu.NS_ARR_CV), ins):
            gs.set(a, x)
        sums = gs.kernel(gpu.NS_K_RHS)
        outs.append([gs.get(a) for a in (gpu.NS_ARR_RU, gpu.NS_ARR_RV, gpu.NS_ARR_CU, gpu.NS_ARR_CV)] + [sums[:2]])
        gs.close()
    for a, b in zip(outs[0][:4], outs[1][:4]):
        assert rel(a, b) <= 1e-14
    np.testing.assert_allclose(outs[0][4], outs[1][4], rtol=1e-13)


@pytest.mark.parametrize("nx,ny,xr,yr,bc", [(300, 201, 1.002, 0.998, BC_FLOW), (130, 256, -1, -1, BC_CAVITY),
                                            (37, 70, 1.05, -1, BC_CAVITY)])
def test_streaming_k3_k5_equal_grid_kernels(gpu, monkeypatch, nx, ny, xr, yr, bc):
    """K3 / K5 as streaming strips (k_cell_s) = the thread-per-cell kernels (NSGPU_CELL=grid):
    same face weights and divisions, so equal to 1e-14 (FMA contraction may differ); same
    reductions; odd ny (the last pair's padding column) included."""
    rng = np.random.default_rng(37)
    dt = 1e-3
    N = nx * ny
    u, v, phi = (rand(rng, N) for _ in range(3))
    outs = []
    for mode in ("stream", "grid"):
        if mode == "grid":
            monkeypatch.setenv("NSGPU_CELL", "grid")
        _, gs = pair(gpu, nx, ny, dt, 100.0, bc, xr, yr)
        gs.set(gpu.NS_ARR_U, u); gs.set(gpu.NS_ARR_V, v); gs.set(gpu.NS_ARR_PHI, phi)
        sums = gs.kernel(gpu.NS_K_DIV)[:2]
        rp = gs.get(gpu.NS_ARR_RPHI)
        mm = gs.kernel(gpu.NS_K_CORRECT)[:4]
        outs.append((rp, sums, mm, gs.get(gpu.NS_ARR_U), gs.get(gpu.NS_ARR_V)))
        gs.close()
    a, b = outs
    assert rel(a[0], b[0]) <= 1e-14
    np.testing.assert_allclose(a[1], b[1], rtol=1e-12, atol=1e-12 * np.abs(b[1]).max())
    np.testing.assert_array_equal(a[2], b[2]) if rel(a[3], b[3]) == 0 else np.testing.assert_allclose(a[2], b[2], rtol=1e-14)
    assert rel(a[3], b[3]) <= 1e-14 and rel(a[4], b[4]) <= 1e-14


def test_step_async_equals_step(gpu):
    """ns_step_async is ns_step without the closing host sync: the same fields bit for bit, and
    its monitor values are the previous step's (ns_monitor returns the latest)."""
    n, dt, re = 96, 1.0 / 768, 400.0
    a = gpu.GpuSolver(gpu.cavity(n), dt, re)
    b = gpu.GpuSolver(gpu.cavity(n), dt, re)
    sync = [a.step() for _ in range(6)]
    lag = [b.step_async() for _ in range(6)]
    assert all(np.isnan(lag[0][k]) for k in ("umin", "umax", "vmin", "vmax"))
    for k in range(1, 6):
        assert [lag[k][q] for q in ("umin", "umax", "vmin", "vmax")] == \
               [sync[k - 1][q] for q in ("umin", "umax", "vmin", "vmax")], k
        assert (lag[k]["it_u"], lag[k]["it_phi"]) == (sync[k]["it_u"], sync[k]["it_phi"])
    assert b.monitor() == (sync[5]["umin"], sync[5]["umax"], sync[5]["vmin"], sync[5]["vmax"])
    with pytest.raises(gpu.NsError):
        b.monitor()   # nothing pending
    for x, y in zip(a.fields(), b.fields()):
        assert np.array_equal(x, y)
    # a synchronous step after async ones continues the same trajectory
    assert a.step()["umax"] == b.step()["umax"]


@pytest.mark.parametrize("n", [96, 512])
def test_deferred_correction_is_bit_identical(gpu, monkeypatch, n):
    """(r6) ns_step_async defers CorrectVelocities (FluidSolver.cpp:512-534) into the next step's K1 (k_rhs_sc:
    u = u* - dt grad phi formed on the fly from u*, v*, phi^n with K5's own arithmetic, corr1), so an async step
    ends after its Poisson solve; reading the fields, the monitor or a synchronous step applies a pending
    correction first (K5).  Against NSGPU_K5_DEFER=0 (K5 at every step's end): the same monitors, sweep counts and
    fields bit for bit -- also across a mid-run field read and an async -> sync -> async switch."""
    dt, re = 1.0 / (8 * n), 400.0
    out = {}
    for d in ("1", "0"):
        monkeypatch.setenv("NSGPU_K5_DEFER", d)
        gs = gpu.GpuSolver(gpu.cavity(n), dt, re)
        st = [gs.step_async() for _ in range(4)]
        mid = [a.copy() for a in gs.fields()]          # (a pending correction applied here)
        st += [gs.step_async() for _ in range(3)]
        st += [gs.step()]                              # (async -> sync)
        st += [gs.step_async() for _ in range(3)]
        last = gs.monitor()
        out[d] = (st, mid, [a.copy() for a in gs.fields()], last)
        gs.close()
    (sa, ma, fa, la), (sb, mb, fb, lb) = out["1"], out["0"]
    key = ("umin", "umax", "vmin", "vmax", "it_u", "it_phi")
    for x, y in zip(sa, sb):
        assert all((np.isnan(x[k]) and np.isnan(y[k])) or x[k] == y[k] for k in key), (x, y)
    assert la == lb
    for x, y in zip(ma + fa, mb + fb):
        assert np.array_equal(x, y)
    # the deferral ran: every async step after the first of a run folded its predecessor's K5 into K1
    assert [x["k5_deferred"] for x in sa] == [0, 1, 1, 1, 0, 1, 1, 0, 0, 1, 1], [x["k5_deferred"] for x in sa]
    assert all(x["k5_deferred"] == 0 for x in sb)


@pytest.mark.parametrize("nx,ny", [(96, 96), (200, 136), (512, 512), (130, 1000)])
def test_band6_is_bit_identical(gpu, monkeypatch, nx, ny):
    """(r6) one rank's 6 wall-band sweeps in ONE launch (k_helm_band6: 64 x 64 tiles, their 12-cell cone staged in
    LDS, the band cells copied back) against two launches of 3 sweeps on 32 x 32 tiles (NSGPU_BAND6=0): a band
    cell's value after 6 RB-SOR sweeps does not depend on the tiling, so the monitors, sweep counts and fields
    agree bit for bit -- grids that are no multiple of 64, bands wider than half a tile row."""
    dt, re = 1.0 / (8 * max(nx, ny)), 400.0
    out = {}
    for d in ("1", "0"):
        monkeypatch.setenv("NSGPU_BAND6", d)
        gs = gpu.GpuSolver(gpu.rectangle(nx, ny), dt, re)
        st = [gs.step() for _ in range(5)]
        out[d] = (st, [a.copy() for a in gs.fields()])
        gs.close()
    (sa, fa), (sb, fb) = out["1"], out["0"]
    key = ("umin", "umax", "vmin", "vmax", "it_u", "it_phi")
    for x, y in zip(sa, sb):
        assert all(x[k] == y[k] for k in key), (x, y)
    for x, y in zip(fa, fb):
        assert np.array_equal(x, y)


def test_known_answer_trace_128_async(gpu):
    """The reference's printed 128^2 monitor through ns_step_async (one step late)."""
    n = 128
    gs = gpu.GpuSolver(gpu.cavity(n), 1.0 / 1024, 100.0)
    for it in range(1, 202):
        st = gs.step_async() if it <= 200 else None
        got = gs.monitor() if it == 201 else (st["umin"], st["umax"], st["vmin"], st["vmax"])
        if it - 1 in KNOWN_TRACE_128:
            assert all(printed_equal(x, y) for x, y in zip(got, KNOWN_TRACE_128[it - 1])), (it - 1, got)


def test_dispatch_stamped_kernel_timing(gpu, monkeypatch):
    """Timed launches use hipExtLaunchKernel's begin / end stamps (the kernel's own interval,
    what rocprofv3 reports); NSGPU_EXT_TIMING=0 brackets them with marker events, which also
    count the dispatch latency.  Both are positive; the dispatch-stamped interval is not longer;
    step timings stay positive and per-pass."""
    n = 1024
    avg = {}
    monkeypatch.setenv("NSGPU_FPS", "0")   # (the multigrid's timed passes)
    for ext in ("1", "0"):
        monkeypatch.setenv("NSGPU_EXT_TIMING", ext)
        js = gpu.GpuSolver(gpu.cavity(n), 1.0 / (8 * n), 1000.0, poisson=gpu.NS_POISSON_JACOBI, omega=1.0)
        js.fill_random(0x5EED)
        avg[ext] = min(js.time_poisson(5, 20)["avg_ms"] for _ in range(3))
        js.close()
        gs = gpu.GpuSolver(gpu.cavity(2 * n), 1.0 / (16 * n), 1000.0, timing=True)
        st = [gs.step() for _ in range(3)]
        assert all(s["n_helm_kernels"] > 0 and s["t_helm_kernel_ms"] > 0 for s in st)
        assert all(s["n_restrict_kernels"] > 0 and s["t_restrict_kernel_ms"] > 0 for s in st)
        gs.close()
    assert 0 < avg["1"] <= avg["0"] * 1.02, avg


@pytest.mark.parametrize("n", [256, 1024])
def test_speculative_correction_is_bit_identical(gpu, monkeypatch, n):
    """The step's K5 (CorrectVelocities, FluidSolver.cpp:512-534) is enqueued behind the
    multigrid's predicted residual check, before the host reads the residual; a check that
    fails discards it.  NSGPU_SPECULATE=0 runs K5 after the solve instead: the same cycles,
    so the fields and monitors must be bit-identical."""
    dt, re = 1.0 / (8 * n), 1000.0
    out = []
    for spec in ("1", "0"):
        monkeypatch.setenv("NSGPU_SPECULATE", spec)
        gs = gpu.GpuSolver(gpu.cavity(n), dt, re)
        st = [gs.step() for _ in range(12)]
        st += [gs.step_async() for _ in range(3)]
        out.append((gs.fields(), [s["it_phi"] for s in st], [s["n_checks"] for s in st],
                    [[s[k] for k in ("umin", "umax", "vmin", "vmax")] for s in st[:12]], gs.monitor()))
        gs.close()
    (fa, ca, na, ma, la), (fb, cb, nb, mb, lb) = out
    assert ca == cb and na == nb
    assert ma == mb and la == lb
    for x, y in zip(fa, fb):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("n", [256, 1024])
def test_k5_poisson_guess_is_bit_identical(gpu, monkeypatch, n):
    """r4: K5 forms the next step's Poisson guess (the phi extrapolation) in its own pass
    (k_cell_s<6>, opt-in: NSGPU_K5_GUESS=1), and K3 runs speculatively behind the Helmholtz residual
    check.  NSGPU_K5_GUESS=0 (the default) is round 3's order (k_axpby at the next step, K3 after the
    check): the same arithmetic, so the
    fields, the V-cycle counts and the monitors must be bit-identical -- through the start-up
    (linear, quadratic, cubic guesses), an injected phi (ns_set_array: the history restarts) and
    a standalone solve between steps (ns_kernel: TMP is overwritten, the guess is formed again)."""
    dt, re = 1.0 / (8 * n), 1000.0
    out = []
    monkeypatch.setenv("NSGPU_FPS", "0")   # (the multigrid's guess: the direct solve takes none)
    for fuse in ("1", "0"):
        monkeypatch.setenv("NSGPU_K5_GUESS", fuse)
        gs = gpu.GpuSolver(gpu.cavity(n), dt, re)
        st = [gs.step() for _ in range(10)]
        phi = gs.get(gpu.NS_ARR_PHI)
        gs.set(gpu.NS_ARR_PHI, phi)
        st += [gs.step() for _ in range(4)]
        rp = gs.get(gpu.NS_ARR_RPHI)
        gs.kernel(gpu.NS_K_RESIDUAL)
        gs.set(gpu.NS_ARR_RPHI, rp)
        st += [gs.step_async() for _ in range(4)]
        out.append((gs.fields(), [s["it_phi"] for s in st], [s["it_u"] for s in st],
                    [[s[k] for k in ("umin", "umax", "vmin", "vmax")] for s in st[:14]], gs.monitor()))
        gs.close()
    (fa, ca, ha, ma, la), (fb, cb, hb, mb, lb) = out
    assert ca == cb and ha == hb
    assert ma == mb and la == lb
    for x, y in zip(fa, fb):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("knob,ran", [("NSGPU_FUSE4", "n_cycle_kernels"), ("NSGPU_GIN", "n_guess_kernels")])
@pytest.mark.parametrize("n,xr", [(256, -1), (2048, -1), (512, 1.002)])
def test_fused_cycle_boundary_is_bit_identical(gpu, monkeypatch, n, xr, knob, ran):
    """r4, NSGPU_FUSE4: a V-cycle whose output is not checked hands its finest prolongation pass to
    the next cycle's restriction pass, one k_sweep4 pass (prolongation + four RB sweeps + residual +
    restriction).  NSGPU_GIN: the solve's first restriction pass forms the phi extrapolation from
    the history planes as rows enter it (k_sweep2_gin) instead of reading k_axpby's guess, and K3
    runs speculatively behind the Helmholtz check.  =0 runs round 3's passes: the same arithmetic
    in the same order, so fields, V-cycle counts and monitors must be bit-identical (uniform and
    stretched rows: the UNI and general instantiations), and the timed passes show each ran.
    (Below 2048^2 the finest level is LDS-tiled; NSGPU_PAIR_MIN_CELLS=0 streams it.)"""
    dt, re = 1.0 / (8 * n), 1000.0
    monkeypatch.setenv("NSGPU_FPS", "0")
    if n < 2048:
        monkeypatch.setenv("NSGPU_PAIR_MIN_CELLS", "0")
    out = []
    for fuse in ("1", "0"):
        monkeypatch.setenv(knob, fuse)
        gs = gpu.GpuSolver(gpu.rectangle(n, n, bc=BC_CAVITY, xratio=xr, yratio=xr), dt, re, timing=True)
        st = [gs.step() for _ in range(12)]
        out.append((gs.fields(), [s["it_phi"] for s in st], [s["n_checks"] for s in st],
                    [[s[k] for k in ("umin", "umax", "vmin", "vmax")] for s in st], sum(s[ran] for s in st)))
        gs.close()
    (fa, ca, na, ma, ka), (fb, cb, nb, mb, kb) = out
    assert ca == cb and na == nb and ma == mb
    assert ka > 0 and kb == 0, (ka, kb)   # (the fused run had cycles whose output went unchecked)
    for x, y in zip(fa, fb):
        assert np.array_equal(x, y)


BC_OUT_W = [(4, 0.0), (2, 0.0), (0, -1.0), (2, 0.0)]     # inflow from E, NEUMANN outflow W


@pytest.mark.parametrize("nx,ny,bc,xr,yr", [(256, 64, BC_CHANNEL, -1, -1), (128, 96, BC_OUT_W, -1, -1),
                                            (512, 128, BC_CHANNEL, -1, -1), (160, 48, BC_CHANNEL, 1.01, 0.98),
                                            (96, 40, BC_OUT_W, 0.99, -1)])
def test_outflow_line_preconditioner(gpu, monkeypatch, nx, ny, bc, xr, yr):
    """A W or E NEUMANN outflow side (FluidSolver.cpp:98-101): the Poisson BiCGStab is
    preconditioned by the outflow side's 1-D line solve (the linear-extrapolation closure's
    decoupled column), extended along x as the initial iterate of a V-cycle whose hierarchy closes
    that side by face-Dirichlet data.  From a random rhs on these anisotropic /
    graded grids it converges (rtol 1e-8) in fewer iterations than the round-1 wall-closure V-cycle
    (NSGPU_OUTFLOW_PC=wall) and in at most 25 (square cells: test_outflow_channel_steps); at rtol
    1e-11 it reaches the oracle's direct solve of the same mean-projected system to 1e-8 relative
    (phi modulo its mean).  (r5: uniform E-outflow channels take the direct solve by default;
    NSGPU_FPS_OUTFLOW=0 keeps them on this Krylov path.)"""
    monkeypatch.setenv("NSGPU_FPS_OUTFLOW", "0")
    rng = np.random.default_rng(12)
    its = {}
    b = rand(rng, nx * ny, 100.0)
    for pc in ("line", "wall"):
        monkeypatch.setenv("NSGPU_OUTFLOW_PC", pc)
        og, gs = pair(gpu, nx, ny, 1.0 / 256, 100.0, bc, xr, yr, rtol=1e-8)
        gs.set(gpu.NS_ARR_PHI, np.zeros(nx * ny)); gs.set(gpu.NS_ARR_RPHI, b)
        n, res = gs.kernel(gpu.NS_K_POIS_SOLVE)[:2]
        its[pc] = n
        assert res <= 1e-8, (pc, n, res)
        gs.close()
    assert its["line"] <= 25, its
    # the solution: the line-closure solve at rtol 1e-11 against the oracle's direct solve (the
    # error of a residual-converged iterate grows with the condition number of these anisotropic
    # grids: rtol 1e-8 left 1.1e-6 at 512 x 128)
    monkeypatch.setenv("NSGPU_OUTFLOW_PC", "line")
    og, gs = pair(gpu, nx, ny, 1.0 / 256, 100.0, bc, xr, yr, rtol=1e-11)
    gs.set(gpu.NS_ARR_PHI, np.zeros(nx * ny)); gs.set(gpu.NS_ARR_RPHI, b)
    n, res = gs.kernel(gpu.NS_K_POIS_SOLVE)[:2]
    xp, _ = og.solve_poisson(b)
    g = gs.get(gpu.NS_ARR_PHI).ravel()
    err = float(rel(g - g.mean(), xp - xp.mean()))
    assert err <= 1e-8, (err, n)
    gs.close()
    assert its["line"] < its["wall"], its


@pytest.mark.parametrize("nx,ny", [(1024, 256), (2048, 512)])
def test_outflow_channel_steps(gpu, monkeypatch, nx, ny):
    """The channel of tools/bench_bcs.py (square cells, inlet W, NEUMANN outflow E, Re 1000) from
    rest: the line-closure preconditioner holds the Poisson BiCGStab to <= 8 iterations per step
    on average (VERDICT r1's target; the wall closure needs 30-60 here), every solve converged.
    (r6, ADVICE r5: these uniform E-outflow channels take the direct solve by default since r5 --
    NSGPU_FPS_OUTFLOW=0 keeps the step on the line-closure Krylov path this test is about; every
    solve there is checked, so res_phi is a real residual, never the unchecked -1.)"""
    monkeypatch.setenv("NSGPU_FPS_OUTFLOW", "0")
    h = 4.0 / nx
    g = gpu.rectangle(nx, ny, lx=4.0, ly=ny * h, bc=BC_CHANNEL)
    gs = gpu.GpuSolver(g, h / 8, 1000.0)
    st = [gs.step() for _ in range(8)]
    gs.close()
    its = [x["it_phi"] for x in st]
    assert min(its) >= 2, its   # a Krylov solve, not the one-shot direct solve
    assert np.mean(its) <= 8.0 and max(its) <= 10, its
    res = [x["res_phi"] for x in st]
    assert all(0.0 <= r <= 1e-8 for r in res), res


def test_outflow_channel_direct_steps_checked(gpu):
    """(r6) The same channel on its default path, the direct solve with the outflow row eliminated: a res_phi bound
    only counts on the solves that were checked (phi_checked 1; the unchecked ones report -1 and are excluded, so
    the sentinel can never satisfy the bound), and the first solve is always checked."""
    nx, ny = 1024, 256
    h = 4.0 / nx
    g = gpu.rectangle(nx, ny, lx=4.0, ly=ny * h, bc=BC_CHANNEL)
    gs = gpu.GpuSolver(g, h / 8, 1000.0)
    st = [gs.step() for _ in range(8)]
    gs.close()
    assert all(x["it_phi"] == 1 for x in st), [x["it_phi"] for x in st]
    checked = [x for x in st if x["phi_checked"]]
    assert st[0]["phi_checked"] == 1 and checked
    assert all(0.0 <= x["res_phi"] <= 1e-8 for x in checked), [x["res_phi"] for x in checked]
    assert all(x["res_phi"] == -1.0 for x in st if not x["phi_checked"])


@pytest.mark.parametrize("nx,ny,bc", [(40, 24, BC_CHANNEL), (24, 48, BC_OUT_N), (30, 26, BC_OUT_WS),
                                      (33, 20, BC_CHANNEL), (200, 134, BC_OUT_WS), (512, 130, BC_OUT_W)])
def test_streaming_poisson_apply_matches_grid_kernel(gpu, monkeypatch, nx, ny, bc):
    """The rectangle's BiCGStab applies LHS_phi (FluidSolver.cpp:105-163, the NEUMANN ghost
    2.5 / -2 / 0.5 of :98-101 on every outflow side) with the streaming strip kernel
    (k_cell_s<7>); NSGPU_CELL=grid is the thread-per-cell k_apply it replaced.  Same solve from
    the same rhs: iteration counts within one and phi within 1e-8 relative at rtol 1e-10 (the strips'
    partial sums group the dot products differently), at the oracle's direct solve (1e-8)."""
    rng = np.random.default_rng(21)
    b = rand(rng, nx * ny, 100.0)
    out = {}
    for mode in ("grid", "stream"):
        if mode == "grid":
            monkeypatch.setenv("NSGPU_CELL", "grid")
        else:
            monkeypatch.delenv("NSGPU_CELL", raising=False)
        og, gs = pair(gpu, nx, ny, 1.0 / 256, 100.0, bc, rtol=1e-10)
        gs.set(gpu.NS_ARR_PHI, np.zeros(nx * ny)); gs.set(gpu.NS_ARR_RPHI, b)
        its, res = gs.kernel(gpu.NS_K_POIS_SOLVE)[:2]
        assert res <= 1e-10, (mode, its, res)
        g = gs.get(gpu.NS_ARR_PHI).ravel()
        out[mode] = (int(its), g - g.mean())
        gs.close()
    assert abs(out["grid"][0] - out["stream"][0]) <= 1, (out["grid"][0], out["stream"][0])
    assert float(rel(out["stream"][1], out["grid"][1])) <= 1e-8
    xp, _ = og.solve_poisson(b)
    assert float(rel(out["stream"][1], xp - xp.mean())) <= 1e-8
