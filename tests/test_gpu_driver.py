"""End to end through the drop-in boundary on the GPU: the repo's ns_main and the
reference's own MAIN_Solver.cpp (compiled unchanged against include/, binary
ref_main_link built where /root/reference exists) read the reference's two input files,
print the reference's monitor and write FlowData_<iter>.csv; all checked against the oracle.
Tolerances: monitor = printf("%lf") digits (last-digit flip allowed); CSV = 6 significant
digits (ostream default, half-unit 5e-6 relative) plus the rtol-1e-8 solve difference
(~1e-7) -> 1e-5 relative + 1e-6 absolute."""
import os
import subprocess

import numpy as np
import pytest

from conftest import printed_equal
from oracle import OGrid, OSolver

pytestmark = pytest.mark.gpu
HOST = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "navierstokessolver_amd", "host")

N, RE, STEPS, SAVE = 32, 100.0, 20, 10
DT = 1.0 / (8 * N)


def write_inputs(d):
    (d / "grid").write_text(f"Vertices {{\n0 0\n0 1\n1 1\n1 0\n}}\nNx {{\n0 1 {N} -1\n}}\nNy {{\n0 1 {N} -1\n}}\n")
    (d / "sim").write_text(f"BC {{\n2 0\n2 1\n2 0\n2 0\n}}\ndt {DT!r}\nfinal_time {STEPS * DT!r}\nre {RE!r}\nsaveIter {SAVE}\n")


@pytest.fixture(scope="module")
def oracle_run():
    og = OGrid.rectangle(N, N)
    s = OSolver(og, DT, RE, rtol=1e-13)
    trace, snaps = [], {}
    for it in range(1, STEPS + 1):
        mm, _ = s.step()
        trace.append(mm)
        if it % SAVE == 0:
            st = s.get()
            snaps[it] = (st["u"], st["v"], og.pressure(DT / (2 * RE), st["phi"]))
    return og, trace, snaps


@pytest.mark.parametrize("exe", ["ns_main", "ref_main_link"])
def test_driver_matches_oracle(tmp_path, exe, oracle_run):
    path = os.path.join(HOST, exe)
    if not os.path.exists(path):
        pytest.skip(f"{exe} not built (ref_main_link needs /root/reference at build time)")
    write_inputs(tmp_path)
    out = subprocess.run([path, "grid", "sim"], capture_output=True, text=True, cwd=tmp_path, timeout=120).stdout
    assert "Solver Setup Complete!" in out and "Solution Complete!" in out, out[-2000:]
    lines = [l for l in out.splitlines() if l and l[0].isdigit()]
    assert len(lines) == STEPS
    og, trace, snaps = oracle_run
    for k, l in enumerate(lines):
        f = l.split("\t")
        assert int(f[0]) == k + 1
        assert all(printed_equal(float(a), b) for a, b in zip(f[1:5], trace[k])), (l, trace[k])
    assert out.count("iter\tumin") == 2   # header every 10 steps
    for it, (u, v, p) in snaps.items():
        d = np.loadtxt(tmp_path / f"FlowData_{it}.csv", delimiter=",", skiprows=1)
        assert d.shape == (N * N + 4 * N, 6)      # one row per cell + one per boundary face
        cells = d[np.isin(np.arange(len(d)), _cell_rows())]
        np.testing.assert_allclose(cells[:, 0], og.xc, atol=1e-6)
        np.testing.assert_allclose(cells[:, 3], u, rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(cells[:, 4], v, rtol=1e-5, atol=1e-6)
        pc = cells[:, 5] - cells[:, 5].mean()
        np.testing.assert_allclose(pc, p - p.mean(), rtol=0, atol=1e-5 * np.abs(p).max())
        top = d[np.isclose(d[:, 1], 1.0)]
        np.testing.assert_allclose(top[:, 3], 1.0, atol=1e-6)   # lid face value u = b (ghost -u + 2b)
        # every boundary-face row (FluidSolver.cpp:596-603): the face point x + nx h/2, the face
        # velocities 0.5 (q + ghost) = c/2 (walls: -q + c, :89-96 -- u = 1 on the lid, 0 elsewhere;
        # v = 0 on every wall) and 0.5 (phi + ghost_phi) - dt/(2 Re) L phi, which for a wall
        # (ghost_phi = phi) is the cell's own Pr
        faces, owner, exp = _face_rows(og)
        fr = d[faces]
        np.testing.assert_allclose(fr[:, 0], exp[:, 0], atol=1e-6)
        np.testing.assert_allclose(fr[:, 1], exp[:, 1], atol=1e-6)
        np.testing.assert_allclose(fr[:, 3], exp[:, 2], atol=1e-12)
        np.testing.assert_allclose(fr[:, 4], exp[:, 3], atol=1e-12)
        np.testing.assert_allclose(fr[:, 5], d[owner, 5], rtol=1e-5, atol=1e-12)
        np.testing.assert_allclose(fr[:, 5] - cells[:, 5].mean(), p[owner_cells(owner)] - p.mean(), rtol=0,
                                   atol=1e-5 * np.abs(p).max())
    assert (tmp_path / "CellCenters.csv").exists()


def _cell_rows():
    # rows are written cell by cell (i outer, j inner), each followed by its boundary faces
    rows, r = [], 0
    for i in range(N):
        for j in range(N):
            rows.append(r)
            r += 1 + (i == 0) + (i == N - 1) + (j == 0) + (j == N - 1)
    return rows


def _face_rows(og):
    """Row indices of the boundary-face rows, the row of the cell each belongs to, and the
    expected (x, y, u, v) of each: faces follow their cell in Cell::edges order W, E, S, N
    (Grid.h:33); the cavity's lid (N side) has u = 1, every other wall 0."""
    h = 1.0 / N
    faces, owner, exp, r = [], [], [], 0
    for i in range(N):
        for j in range(N):
            cell = r
            r += 1
            xc, yc = (i + 0.5) * h, (j + 0.5) * h
            for on, (nx, ny) in zip((i == 0, i == N - 1, j == 0, j == N - 1), ((-1, 0), (1, 0), (0, -1), (0, 1))):
                if not on:
                    continue
                faces.append(r)
                owner.append(cell)
                exp.append((xc + nx * h / 2, yc + ny * h / 2, 1.0 if ny == 1 else 0.0, 0.0))
                r += 1
    return np.array(faces), np.array(owner), np.array(exp)


def owner_cells(owner_rows):
    """Cell index (compact id order) of each owner row."""
    idx = {row: k for k, row in enumerate(_cell_rows())}
    return np.array([idx[r] for r in owner_rows])


# ---- a backward-facing step with an inlet and a NEUMANN outflow (tests/polygons.py STEP):
# the host Grid classifies the polygon, FluidSolver hands libnsgpu.so the mask, the export
# includes the outflow's ghost rows in L phi (MatMult(LHS_phi), FluidSolver.cpp:579)
from polygons import STEP  # noqa: E402

PSTEPS, PSAVE = 12, 6


def write_polygon_inputs(d, P, dt):
    verts = "\n".join(f"{x} {y}" for x, y in P["vertices"])
    seg = lambda spec: "\n".join(" ".join(str(v) for v in s) for s in spec)
    (d / "grid").write_text(f"Vertices {{\n{verts}\n}}\nNx {{\n{seg(P['xspec'])}\n}}\nNy {{\n{seg(P['yspec'])}\n}}\n")
    bc = "\n".join(f"{t} {i}" for t, i in P["bc"])
    (d / "sim").write_text(f"BC {{\n{bc}\n}}\ndt {dt!r}\nfinal_time {PSTEPS * dt!r}\nre {RE!r}\nsaveIter {PSAVE}\n")


@pytest.mark.parametrize("exe", ["ns_main", "ref_main_link"])
def test_driver_polygon_outflow_matches_oracle(tmp_path, exe):
    path = os.path.join(HOST, exe)
    if not os.path.exists(path):
        pytest.skip(f"{exe} not built (ref_main_link needs /root/reference at build time)")
    P = STEP
    dt = 1.0 / 512
    write_polygon_inputs(tmp_path, P, dt)
    out = subprocess.run([path, "grid", "sim"], capture_output=True, text=True, cwd=tmp_path, timeout=120).stdout
    assert "Solver Setup Complete!" in out and "Solution Complete!" in out, out[-2000:]
    lines = [l for l in out.splitlines() if l and l[0].isdigit()]
    assert len(lines) == PSTEPS
    og = OGrid(P["vertices"], P["xspec"], P["yspec"], P["bc"])
    osv = OSolver(og, dt, RE, rtol=1e-13)
    tags = og.tag.reshape(og.nx, og.ny, 4)
    ids = og.id.reshape(og.nx, og.ny)
    rows, r = [], 0          # each in-domain cell's row, then one row per boundary face
    for i in range(og.nx):
        for j in range(og.ny):
            if ids[i, j] < 0:
                continue
            rows.append(r)
            r += 1 + int((tags[i, j] >= 0).sum())
    for it in range(1, PSTEPS + 1):
        mm, _ = osv.step()
        f = lines[it - 1].split("\t")
        assert all(printed_equal(float(a), b) for a, b in zip(f[1:5], mm)), (lines[it - 1], mm)
        if it % PSAVE:
            continue
        st = osv.get()
        d = np.loadtxt(tmp_path / f"FlowData_{it}.csv", delimiter=",", skiprows=1)
        assert d.shape == (r, 6)
        cells = d[rows]
        np.testing.assert_allclose(cells[:, 0], og.xc, atol=1e-5)   # 6 significant digits, x up to 2
        np.testing.assert_allclose(cells[:, 1], og.yc, atol=1e-5)
        np.testing.assert_allclose(cells[:, 3], st["u"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(cells[:, 4], st["v"], rtol=1e-5, atol=1e-6)
        p = og.pressure(dt / (2 * RE), st["phi"])
        pc = cells[:, 5] - cells[:, 5].mean()
        np.testing.assert_allclose(pc, p - p.mean(), rtol=0, atol=1e-5 * np.abs(p).max())
