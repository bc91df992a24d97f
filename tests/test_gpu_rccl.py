"""The RCCL call sites of libnsgpu.so on MI355X with one GPU (they had never run).

NSGPU_RCCL_LOOPBACK=1 gives a one-rank solver a 1-rank RCCL communicator: every exchange
point of the step runs its ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd group
(halo_reqs, ns_solver.cpp) with peer == self -- both ghost sides filled from the slab's own
edge rows, on the comm stream of the overlapped passes -- and every reduction runs
ncclAllReduce.  Ghost rows beyond a wall carry zero weight in every kernel, so the step must
be the plain single-rank step: fields bit-identical, the same sweep / V-cycle counts.  The
exchange and all-reduce counters (ns_stats.n_exchanges / n_allreduces) prove the RCCL
branch ran.  (What one GPU cannot show: xGMI transfers between two devices.)"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def run(gpu, monkeypatch, grid, dt, re, steps, loopback, overlap=True, **kw):
    monkeypatch.setenv("NSGPU_RCCL_LOOPBACK", "1" if loopback else "0")
    monkeypatch.setenv("NSGPU_OVERLAP", "1" if overlap else "0")
    gs = gpu.GpuSolver(grid, dt, re, device=0, **kw)
    monkeypatch.delenv("NSGPU_RCCL_LOOPBACK")
    st = [gs.step() for _ in range(steps)]
    u, v, phi = gs.fields()
    gs.close()
    return u, v, phi, st


def counts(st):
    return [(s["it_u"], s["it_v"], s["it_phi"]) for s in st]


@pytest.mark.parametrize("case", ["cavity_mg", "cavity_mg_no_overlap", "channel_outflow", "lshape"])
def test_rccl_loopback_step_equals_single_rank(gpu, monkeypatch, case):
    if case.startswith("cavity"):
        n = 256
        grid, dt, re = gpu.cavity(n), 1.0 / (8 * n), 1000.0
    elif case == "channel_outflow":
        grid = gpu.rectangle(128, 64, lx=2.0, ly=1.0, bc=[(0, 1.0), (2, 0.0), (4, 0.0), (2, 0.0)])
        dt, re = 1.0 / 512, 100.0
    else:
        from polygons import ALL
        P = ALL["lshape"]
        from oracle import OGrid
        og = OGrid(P["vertices"], P["xspec"], P["yspec"], P["bc"])
        grid, dt, re = gpu.polygon(P["vertices"], og.hx, og.hy, P["bc"]), 1.0 / 1024, 200.0
    overlap = case != "cavity_mg_no_overlap"
    a = run(gpu, monkeypatch, grid, dt, re, 4, False)
    b = run(gpu, monkeypatch, grid, dt, re, 4, True, overlap=overlap)
    assert all(s["n_exchanges"] == 0 and s["n_allreduces"] == 0 and s["x_link_bytes"] == 0 for s in a[3])
    assert all(s["x_link_bytes"] > 0 for s in b[3])
    assert all(s["n_exchanges"] > 0 and s["n_allreduces"] > 0 for s in b[3]), [
        (s["n_exchanges"], s["n_allreduces"]) for s in b[3]]
    assert counts(a[3]) == counts(b[3])
    for x, y in zip(a[:3], b[:3]):
        assert np.array_equal(x, y), float(np.max(np.abs(x - y)))
    mm_a = [[s[k] for k in ("umin", "umax", "vmin", "vmax")] for s in a[3]]
    mm_b = [[s[k] for k in ("umin", "umax", "vmin", "vmax")] for s in b[3]]
    assert mm_a == mm_b


def test_virtual_slab_replays_counts(gpu, monkeypatch):
    """A virtual slab (NSGPU_RCCL_LOOPBACK with nranks > 1, no ncclUniqueId): rank 2 of 4 builds
    its slab and hierarchy and runs every RCCL group with itself as the peer; each step replays
    the given (Helmholtz sweeps, V-cycles) -- tools/slab_projection.py's per-rank timing.  It
    must run those counts exactly, issue exchanges and all-reduces (and the agglomeration
    gather: the level hierarchy has replicated levels at 4 ranks), and stay finite."""
    n = 512
    monkeypatch.setenv("NSGPU_FPS", "0")   # (the multigrid's replayed cycles; the direct solve's: below)
    monkeypatch.setenv("NSGPU_RCCL_LOOPBACK", "1")
    monkeypatch.setenv("NSGPU_VIRTUAL_ITERS", "4:2,6:3")
    gs = gpu.GpuSolver(gpu.cavity(n), 1.0 / (8 * n), 1000.0, device=0, rank=2, nranks=4)
    st = [gs.step() for _ in range(4)]
    u, v, _ = gs.fields()
    gs.close()
    assert [(s["it_u"], s["it_phi"]) for s in st] == [(4, 2), (6, 3), (4, 2), (6, 3)]
    assert all(s["n_exchanges"] > 0 and s["n_allreduces"] > 0 for s in st)
    # ns_stats.x_link_bytes (ABI 5): at least this rank's slab of the replicated 256^2 level per
    # V-cycle (the agglomeration gather: 64 of its rows) plus ghost rows
    assert all(s["x_link_bytes"] >= s["it_phi"] * (n // 8) * (n // 2) * 8 for s in st), [s["x_link_bytes"] for s in st]
    assert np.all(np.isfinite(u)) and np.all(np.isfinite(v)) and u.shape == (n // 4, n)
    monkeypatch.delenv("NSGPU_VIRTUAL_ITERS")
    with pytest.raises(gpu.NsError):   # a virtual slab without replayed counts would never converge
        gpu.GpuSolver(gpu.cavity(n), 1.0 / (8 * n), 1000.0, device=0, rank=2, nranks=4)


def test_virtual_slab_direct_solve(gpu, monkeypatch):
    """The direct Poisson solve on a virtual slab (rank 2 of 4): one solve per step (it_phi 1), the
    two per-direction allgathers of the ranks' recurrence aggregates counted as collectives and their
    bytes on the link, finite fields."""
    n = 512
    monkeypatch.setenv("NSGPU_RCCL_LOOPBACK", "1")
    monkeypatch.setenv("NSGPU_VIRTUAL_ITERS", "4:1")
    gs = gpu.GpuSolver(gpu.cavity(n), 1.0 / (8 * n), 1000.0, device=0, rank=2, nranks=4)
    st = [gs.step() for _ in range(3)]
    u, v, _ = gs.fields()
    gs.close()
    assert [(s["it_u"], s["it_phi"]) for s in st] == [(4, 1)] * 3
    assert all(s["n_allreduces"] >= 2 and s["x_link_bytes"] >= 2 * 2 * n * 8 for s in st)
    assert np.all(np.isfinite(u)) and np.all(np.isfinite(v))
