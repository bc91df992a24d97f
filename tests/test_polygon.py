"""Non-rectangular domains, host side (no GPU): the Python polygon classifier that feeds
ns_create's cell_id / face_edge equals the oracle's restatement of Grid.cpp:131-185."""
import numpy as np
import pytest

import navierstokessolver_amd as nsa
from oracle import OGrid
from polygons import ALL


@pytest.mark.parametrize("name", sorted(ALL))
def test_polygon_classifier_matches_oracle(name):
    P = ALL[name]
    og = OGrid(P["vertices"], P["xspec"], P["yspec"], P["bc"])
    gs = nsa.polygon(P["vertices"], og.hx, og.hy, P["bc"])
    assert gs.cell_id is not None
    np.testing.assert_array_equal(gs.cell_id, og.id)
    np.testing.assert_array_equal(gs.face_edge, og.tag)
    assert int(gs.mask.sum()) == og.N
    assert [(e.nx, e.ny) for e in gs.edges] == [
        ((-1 if b[1] > a[1] else 1), 0) if a[0] == b[0] else (0, (1 if b[0] > a[0] else -1))
        for a, b in zip(P["vertices"], P["vertices"][1:] + P["vertices"][:1])]


def test_polygon_rectangle_is_the_fast_path():
    gs = nsa.polygon([(0, 0), (0, 1), (1, 1), (1, 0)], np.full(8, 0.125), np.full(8, 0.125), [(2, 0.0)] * 4)
    assert gs.cell_id is None and gs.face_edge is None
