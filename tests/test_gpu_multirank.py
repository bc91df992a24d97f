"""Multi-rank (x-slab) path with the real kernels: 2 processes on one GPU exchanging ghost
rows through the host transport (libnsgpu.so's RCCL call sites swapped for host
callbacks).  The gathered slabs must equal the single-rank run: bit-for-bit for the
RB-SOR solver up to the stopping decision (sweeps are decomposition-independent),
within solver tolerance for multigrid (its hierarchy is cut earlier on slabs).
Also probes whether RCCL accepts two ranks on one device (it normally refuses)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import navierstokessolver_amd as nsa

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(autouse=True)
def _multigrid(monkeypatch):
    """These tests check the multigrid slab protocol (hierarchy, agglomeration, overlapped
    exchanges): the single-rank reference runs the multigrid too (NSGPU_FPS=0; the direct solve's
    slabs: test_gpu_fps.py)."""
    monkeypatch.setenv("NSGPU_FPS", "0")


def launch(tmp_path, *args, port=29561, nproc=2):
    out = tmp_path / "r.npz"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(HERE, "mr_worker.py"),
           "--output", str(out), *args]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=150, env=dict(os.environ))
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    return dict(np.load(out, allow_pickle=False))


def single(n, ny, steps, poisson, rtol, bc=None):
    gs = nsa.GpuSolver(nsa.rectangle(n, ny, bc=bc), 1.0 / (8 * n), 100.0, poisson=poisson, rtol=rtol, device=0)
    mm = [list(gs.step().values())[:7] for _ in range(steps)]
    u, v, phi = gs.fields()
    return u, v, phi, np.array(mm)


@pytest.mark.parametrize("poisson,n,ny,pairs,agg,nproc", [
    (nsa.NS_POISSON_RBSOR, 48, 40, False, None, 2),
    (nsa.NS_POISSON_MG, 64, 64, False, None, 2),
    (nsa.NS_POISSON_MG, 130, 96, False, None, 2),
    (nsa.NS_POISSON_MG, 128, 96, True, None, 2),
    (nsa.NS_POISSON_MG, 128, 96, True, "0", 2),
    (nsa.NS_POISSON_MG, 256, 128, False, "2048", 4),
    (nsa.NS_POISSON_MG, 264, 160, True, "4096", 3),
    (nsa.NS_POISSON_MG, 256, 128, True, None, 3),   # 256 / 3: the old 86/85/85 rows stopped the hierarchy
])
def test_slabs_host_transport_match_single_rank(tmp_path, monkeypatch, poisson, n, ny, pairs, agg, nproc):
    """pairs: every level smoothed by two-sweep passes with the fused restriction (5 ghost rows),
    the path 4096^2 production runs take on their finest levels.  agg: NSGPU_AGG_CELLS, the
    coarse-level agglomeration threshold (None = default 1024^2: every coarse level of these
    grids is replicated; "0" = never, the distributed coarse solve; "2048" = distributed levels
    down to 2048 cells, then the gather onto every rank)."""
    if pairs:
        monkeypatch.setenv("NSGPU_PAIR_MIN_CELLS", "0")
    if agg is not None:
        monkeypatch.setenv("NSGPU_AGG_CELLS", agg)
    steps, rtol = 6, 1e-11
    r = launch(tmp_path, "--xport", "host", "--size", str(n), "--size-y", str(ny), "--nsteps", str(steps),
               "--solver", str(poisson), "--tol", str(rtol), nproc=nproc, port=29561 + nproc)
    assert str(r["status"]) == "ok", r["status"]
    u, v, phi, mm = single(n, ny, steps, poisson, rtol)
    assert r["u"].shape == u.shape
    tol = 1e-9
    assert np.max(np.abs(r["u"] - u)) <= tol
    assert np.max(np.abs(r["v"] - v)) <= tol
    np.testing.assert_allclose(r["mm"][:, :4], mm[:, :4], atol=tol)
    # Helmholtz sweeps per step: the slabs' residual checks see the same residual as the
    # whole grid (a stale ghost row shows up as a solve that never reaches its tolerance)
    assert np.max(np.abs(r["mm"][:, 4] - mm[:, 4])) <= 2, (r["mm"][:, 4], mm[:, 4])
    edges = [nsa.slab_range(n, nproc, q)[0] for q in range(nproc)]
    if poisson == nsa.NS_POISSON_MG and agg != "0" and all(e % 2 == 0 for e in edges) and n % 2 == 0:
        # agglomerated: the same hierarchy as one rank, so the same V-cycle count per step
        assert np.max(np.abs(r["mm"][:, 6] - mm[:, 6])) <= 1, (r["mm"][:, 6], mm[:, 6])


@pytest.mark.parametrize("bc,nproc", [
    ([(0, 1.0), (2, 0.0), (4, 0.0), (2, 0.0)], 2),    # channel: inlet W, outflow E (the last slab)
    ([(4, 0.0), (2, 0.0), (0, -1.0), (2, 0.0)], 3),   # reversed: outflow W (the first slab)
    ([(2, 0.0), (4, 0.0), (2, 0.0), (0, 1.0)], 2),    # outflow N: inside every slab's rows
])
def test_neumann_outflow_slabs_match_single_rank(tmp_path, bc, nproc):
    """NEUMANN outflow (BiCGStab + V-cycle preconditioner): ghost rows before every operator
    application and preconditioner, and every dot product all-reduced -- the slabs converge
    to the single-rank solution."""
    n, ny, steps, rtol = 96, 64, 5, 1e-11
    spec = ",".join(f"{t}:{i}" for t, i in bc)
    r = launch(tmp_path, "--xport", "host", "--size", str(n), "--size-y", str(ny), "--nsteps", str(steps),
               "--solver", str(nsa.NS_POISSON_MG), "--tol", str(rtol), "--bc", spec, nproc=nproc,
               port=29581 + nproc)
    assert str(r["status"]) == "ok", r["status"]
    u, v, phi, mm = single(n, ny, steps, nsa.NS_POISSON_MG, rtol, bc)
    assert np.max(np.abs(r["u"] - u)) <= 1e-8
    assert np.max(np.abs(r["v"] - v)) <= 1e-8
    np.testing.assert_allclose(r["mm"][:, :4], mm[:, :4], atol=1e-8)


@pytest.mark.parametrize("poly,nproc", [("step", 2), ("uchannel", 3)])
def test_masked_domain_slabs_match_single_rank(tmp_path, poly, nproc):
    """Non-rectangular domain on x-slabs: the topology plane carries its ghost rows from the
    global mask, the Krylov solves all-reduce every dot product."""
    from oracle import OGrid
    from polygons import ALL
    P = ALL[poly]
    og = OGrid(P["vertices"], P["xspec"], P["yspec"], P["bc"])
    steps, rtol = 5, 1e-11
    r = launch(tmp_path, "--xport", "host", "--poly", poly, "--nsteps", str(steps), "--tol", str(rtol),
               nproc=nproc, port=29591 + nproc)
    assert str(r["status"]) == "ok", r["status"]
    gs = nsa.GpuSolver(nsa.polygon(P["vertices"], og.hx, og.hy, P["bc"]), 1.0 / (8 * og.nx), 100.0, rtol=rtol,
                       device=0)
    mm = np.array([list(gs.step().values())[:7] for _ in range(steps)])
    u, v, _ = gs.fields()
    du, dv = float(np.max(np.abs(r["u"] - u))), float(np.max(np.abs(r["v"] - v)))
    assert du <= 1e-8 and dv <= 1e-8, (du, dv)
    np.testing.assert_allclose(r["mm"][:, :4], mm[:, :4], atol=1e-8)


def test_stretched_slabs_match_single_rank(tmp_path):
    """Stretched cavity on 2 slabs: the consistent Poisson rhs (area-weighted sums all-reduced)
    and the multigrid on non-uniform spacing give the single-rank answer."""
    n, ny, steps, rtol, ratio = 96, 64, 5, 1e-11, 1.01
    r = launch(tmp_path, "--xport", "host", "--size", str(n), "--size-y", str(ny), "--nsteps", str(steps),
               "--tol", str(rtol), "--ratio", str(ratio), nproc=2, port=29601)
    assert str(r["status"]) == "ok", r["status"]
    gs = nsa.GpuSolver(nsa.rectangle(n, ny, xratio=ratio, yratio=ratio), 1.0 / (8 * n), 100.0, rtol=rtol, device=0)
    mm = np.array([list(gs.step().values())[:7] for _ in range(steps)])
    assert np.all(mm[:, 6] < 100), mm[:, 6]   # V-cycles per step: converging, not stalled
    u, v, _ = gs.fields()
    du, dv = float(np.max(np.abs(r["u"] - u))), float(np.max(np.abs(r["v"] - v)))
    assert du <= 1e-8 and dv <= 1e-8, (du, dv)


@pytest.mark.parametrize("nproc", [2, 3])
def test_overlapped_exchange_is_bit_identical(tmp_path, monkeypatch, nproc):
    """The two-sweep passes' exchange / compute overlap (interior strips while the ghost rows
    travel on the comm stream, then the edge strips) changes no arithmetic: the slabs match a
    run with the plain exchange-then-pass order bit for bit (multigrid and Helmholtz pairs on
    every distributed level, 5-row ghost exchanges, strips of 16 rows)."""
    monkeypatch.setenv("NSGPU_PAIR_MIN_CELLS", "0")
    monkeypatch.setenv("NSGPU_STRIP_ROWS", "16")
    args = ["--xport", "host", "--size", "192", "--size-y", "160", "--nsteps", "4", "--tol", "1e-11"]
    monkeypatch.setenv("NSGPU_OVERLAP", "1")
    a = launch(tmp_path, *args, nproc=nproc, port=29621 + nproc)
    monkeypatch.setenv("NSGPU_OVERLAP", "0")
    b = launch(tmp_path, *args, nproc=nproc, port=29631 + nproc)
    assert str(a["status"]) == "ok" and str(b["status"]) == "ok", (a["status"], b["status"])
    for k in ("u", "v", "phi", "mm"):
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("n,ny,nproc", [(64, 600, 2), (90, 250, 3)])
def test_fp32_jacobi_slabs_match_single_rank(tmp_path, n, ny, nproc):
    """fp32-field Jacobi sweeps (configs[4]) on slabs: the float ghost rows travel as ld/2
    doubles; every cell's update is decomposition-independent, so phi is bit-identical."""
    k = 7
    r = launch(tmp_path, "--xport", "host", "--size", str(n), "--size-y", str(ny), "--sweep32", str(k),
               nproc=nproc, port=29611 + nproc)
    assert str(r["status"]) == "ok", r["status"]
    gs = nsa.GpuSolver(nsa.rectangle(n, ny), 1.0 / (8 * n), 100.0, poisson=nsa.NS_POISSON_JACOBI, omega=0.8, device=0)
    gs.fill_random(0x5EED)
    res = gs.kernel(nsa.NS_K_POISSON32, k)[0]
    phi = gs.fields()[2]
    assert np.array_equal(r["phi"], phi)
    assert abs(r["mm"][0, 0] - res) <= 1e-12 * res


def test_rccl_two_ranks_one_gpu_probe(tmp_path):
    """RCCL usually rejects two ranks on one device; record what it does (never fails the suite
    unless RCCL ran and produced a wrong answer)."""
    try:
        r = launch(tmp_path, "--xport", "rccl", "--size", "48", "--size-y", "40", "--nsteps", "4", "--solver",
                   str(nsa.NS_POISSON_RBSOR), port=29571)
    except (AssertionError, subprocess.TimeoutExpired) as e:
        pytest.skip(f"RCCL two-ranks-on-one-GPU not available here: {str(e)[-300:]}")
    if str(r["status"]) != "ok":
        pytest.skip(f"RCCL refused: {r['status']}")
    u, v, phi, mm = single(48, 40, 4, nsa.NS_POISSON_RBSOR, 1e-10)
    assert np.max(np.abs(r["u"] - u)) <= 1e-9


def test_async_steps_on_slabs_match_sync(tmp_path):
    """ns_step_async on 2 slabs (host transport): the same fields and, realigned by one call,
    the same min/max monitor and iteration counts as ns_step -- bit for bit."""
    args = ["--xport", "host", "--size", "128", "--size-y", "96", "--nsteps", "5", "--tol", "1e-10"]
    a = launch(tmp_path, *args, port=29651)
    b = launch(tmp_path, *args, "--async-steps", port=29653)
    assert str(a["status"]) == "ok" and str(b["status"]) == "ok", (a["status"], b["status"])
    for k in ("u", "v", "phi", "mm"):
        assert np.array_equal(a[k], b[k]), k
