"""Host logic of the drop-in (no GPU): the C++ Grid reads grid files exactly like the
reference's Grid (checked against the oracle's restatement of Grid.cpp), the simulation
file reader / validation follow FluidSolver.cpp's rules, and the reference's own
MAIN_Solver.cpp links unchanged against include/ + libnsfluid.a + libnsgpu.so."""
import json
import os
import subprocess

import numpy as np
import pytest

from oracle import OGrid

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "navierstokessolver_amd", "host")


def run_check(tmp_path, grid_txt, sim_txt=None):
    g = tmp_path / "grid.txt"
    g.write_text(grid_txt)
    args = [os.path.join(HOST, "host_check"), str(g)]
    if sim_txt is not None:
        s = tmp_path / "sim.txt"
        s.write_text(sim_txt)
        args.append(str(s))
    out = subprocess.run(args, capture_output=True, text=True, cwd=tmp_path, check=True).stdout
    js = json.loads(out[out.index("@@JSON") + 6: out.rindex("@@")])
    return js, out


def grid_text(vertices, xs, ys):
    v = "\n".join(f"{a} {b}" for a, b in vertices)
    x = "\n".join(" ".join(str(t) for t in r) for r in xs)
    y = "\n".join(" ".join(str(t) for t in r) for r in ys)
    return f"Vertices {{\n{v}\n}}\nNx {{\n{x}\n}}\nNy {{\n{y}\n}}\n"


CASES = [
    ([(0, 0), (0, 1), (1, 1), (1, 0)], [[0, 1, 8, -1]], [[0, 1, 6, -1]]),
    ([(0, 0), (0, 2), (3, 2), (3, 0)], [[0, 1, 4, -1], [1, 3, 6, 1.2]], [[0, 2, 10, 0.9]]),
    ([(0, 0), (0, 2), (1, 2), (1, 1), (2, 1), (2, 0)], [[0, 2, 8, -1]], [[0, 2, 8, -1]]),   # L-shape
    ([(0, 0), (0, 1), (2, 1), (2, 0)], [[0, 1, 5, -1], [1, 2, 0, -1]], [[0, 1, 5, -1]]),    # count from spacing
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_grid_matches_oracle_restatement(tmp_path, case):
    v, xs, ys = CASES[case]
    js, _ = run_check(tmp_path, grid_text(v, xs, ys))
    og = OGrid(v, xs, ys, [(2, 0.0)] * len(v))
    assert js["setup"]
    assert (js["N"], js["nx"], js["ny"]) == (og.N, og.nx, og.ny)
    np.testing.assert_array_equal(js["hx"], og.hx)
    np.testing.assert_array_equal(js["hy"], og.hy)
    np.testing.assert_array_equal(js["id"], og.id)
    np.testing.assert_array_equal(js["tag"], og.tag)
    assert js["rect"] == (len(v) == 4)
    assert js["cells_table"]
    assert os.path.exists(tmp_path / "CellCenters.csv")
    cc = np.loadtxt(tmp_path / "CellCenters.csv", delimiter=",", ndmin=2)
    np.testing.assert_allclose(cc[:, 0], og.xc, atol=1e-5)   # ostream default precision (6 digits)
    np.testing.assert_allclose(cc[:, 1], og.yc, atol=1e-5)


def test_missing_trailing_values_default_to_uniform(tmp_path):
    js, _ = run_check(tmp_path, "Vertices {\n0 0\n0 1\n1 1\n1 0\n}\nNx {\n0 1 4\n}\nNy {\n0 1 4\n}\n")
    assert js["setup"] and js["N"] == 16


@pytest.mark.parametrize("txt,msg", [
    ("Vertices {\n0 0\n1 0\n1 1\n0 1\n}\nNx {\n0 1 4 -1\n}\nNy {\n0 1 4 -1\n}\n",
     "Invalid specification for number of cells"),                       # counter-clockwise
    ("Vertices {\n0 0\n0 1\n1 2\n1 0\n}\nNx {\n0 1 4 -1\n}\nNy {\n0 1 4 -1\n}\n",
     "Edges should be parallel to the x-axis or y-axis"),
    ("Vertices {\n0 0\n0 1\n1 1\n1 0\n}\nNx {\n0 1 4 -1\n}\nNz {\n0 1 4 -1\n}\n", "Invalid data file format!"),
    ("Vertices {\n0 0\n0 1\n1 1\n1 0\n}\nNx {\n0 1 4 -1\n}\nNy {\n0 0.5 4 -1\n}\n",
     "Invalid specification for number of cells"),
])
def test_invalid_grid_files(tmp_path, txt, msg):
    js, out = run_check(tmp_path, txt)
    assert not js["setup"]
    assert msg in out


SQUARE = "Vertices {\n0 0\n0 1\n1 1\n1 0\n}\nNx {\n0 1 8 -1\n}\nNy {\n0 1 8 -1\n}\n"


def test_sim_file_parsed_like_the_reference(tmp_path):
    js, _ = run_check(tmp_path, SQUARE, "BC {\n2 0\n2 1\n0 0.5\n2 0\n}\ndt 0.001\nfinal_time 0.01\nre 250\nsaveIter 3\n")
    assert js["sim_ok"] and js["sim_valid"] and js["ghosts"]
    assert (js["dt"], js["final_time"], js["re"], js["saveIter"]) == (0.001, 0.01, 250, 3)
    # ghost constants (FluidSolver.cpp:89-96): wall on a horizontal edge -> (2b, 0); inlet on a vertical edge -> (2b, 0)
    assert js["bc"][1] == [2, 1, 2, 0]
    assert js["bc"][2] == [0, 0.5, 1, 0]
    assert js["bc"][0] == [2, 0, 0, 0]


@pytest.mark.parametrize("sim,msg", [
    ("BC {\n2 0\n2 1\n2 0\n2 0\n}\ndt 0.001\nfinal_time 0.01\nre 250\nsaveIter 3", "Invalid data file format!"),  # no trailing ws
    ("BC {\n2 0\n2 1\n2 0\n}\ndt 0.001\nfinal_time 0.01\nre 250\n", "Invalid data file format!"),   # too few BC lines
    ("BC {\n2 0\n2 1\n2 0\n2 0\n}\ndt 0.1\nfinal_time 0.01\nre 250\n", "Time step should be less than final time!"),
    ("BC {\n2 0\n2 1\n2 0\n2 0\n}\ndt 0.001\nfinal_time 0.01\nre -1\n", "Reynolds number should be positive"),
    ("BC {\n2 0\n2 1\n2 0\n2 0\n}\nfinal_time 0.01\nre 10\n", "Time step should be positive"),
    ("BC {\n2 0\n2 1\n2 0\n2 0\n}\ndt 0.001\nfinal_time 0.01\nre 10\nsaveIter 0\n", "saveIter must be greater than zero!"),
    ("BC {\n2 0\n2 1\n2 0\n2 0\n}\ndt 0.001\nfinal_time 0.01\nre 10\nfoo 1\n", "Invalid data file format!"),
])
def test_invalid_sim_files(tmp_path, sim, msg):
    js, out = run_check(tmp_path, SQUARE, sim)
    assert not js["sim_valid"]
    assert msg in out


def test_unsupported_bc_types_rejected(tmp_path):
    js, _ = run_check(tmp_path, SQUARE, "BC {\n1 1\n2 1\n2 0\n2 0\n}\ndt 0.001\nfinal_time 0.01\nre 250\n")
    assert js["sim_valid"] and not js["ghosts"]


@pytest.mark.skipif(not os.path.exists("/root/reference/SRC/MAIN_Solver.cpp"), reason="reference not mounted")
def test_reference_main_links_unchanged(tmp_path):
    exe = os.path.join(HOST, "ref_main_link")
    assert os.path.exists(exe), "navierstokessolver_amd/host/Makefile did not build ref_main_link"
    out = subprocess.run([exe], capture_output=True, text=True, cwd=tmp_path).stdout
    assert "Grid data file or simulation data file not provided!" in out


def test_config_size_grid_stays_compact(tmp_path):
    """configs[3] (8192^2 = 2^26 cells): the rectangle keeps nothing per cell and no
    reference-style `cells` table (~190 B/cell, i.e. ~12 GB at this size); -no_export also
    skips CellCenters.csv (1.2 GB here; Grid.cpp:221-231).  Bound: 64 MB resident."""
    g = tmp_path / "grid.txt"
    g.write_text(grid_text([(0, 0), (0, 1), (1, 1), (1, 0)], [[0, 1, 8192, -1]], [[0, 1, 8192, -1]]))
    out = subprocess.run([os.path.join(HOST, "host_check"), str(g), "-no_export", "-summary"], capture_output=True,
                         text=True, cwd=tmp_path, check=True).stdout
    js = json.loads(out[out.index("@@JSON") + 6: out.rindex("@@")])
    assert js["setup"] and js["rect"] and js["N"] == 8192 * 8192
    assert not js["cells_table"]
    assert 0 < js["maxrss_kb"] < 64 * 1024, js
    assert not os.path.exists(tmp_path / "CellCenters.csv")


def test_cells_table_cap_and_polygon_accessors(tmp_path):
    """The reference-style table is built up to NS_GRID_CELLS_MAX cells (default 2^22) and
    matches the compact accessors; an L-shape keeps its id / tag planes."""
    v, xs, ys = CASES[2]
    js, _ = run_check(tmp_path, grid_text(v, xs, ys))
    assert js["cells_table"] and not js["rect"]
    env = dict(os.environ, NS_GRID_CELLS_MAX="10")
    g = tmp_path / "grid.txt"
    out = subprocess.run([os.path.join(HOST, "host_check"), str(g), "-summary"], capture_output=True, text=True,
                         cwd=tmp_path, check=True, env=env).stdout
    js = json.loads(out[out.index("@@JSON") + 6: out.rindex("@@")])
    assert js["setup"] and not js["cells_table"]
