"""ABI hygiene on the GPU: a zero-initialised ns_params (only dt, re set)
selects the multigrid Poisson solve (ABI 4: NS_POISSON_MG == 0), and the retired value 2 (ABI 3's
NS_POISSON_MG) is rejected loudly instead of silently meaning something else."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _create(L, n, prm):
    hx = np.full(n, 1.0 / n)
    edges = (L.NsEdge * 4)(L.NsEdge(-1, 0, 2, 0.0), L.NsEdge(0, 1, 2, 1.0), L.NsEdge(1, 0, 2, 0.0),
                           L.NsEdge(0, -1, 2, 0.0))
    dp = hx.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    desc = L.NsGridDesc(n, n, dp, dp, 4, edges, None, None)
    h = ctypes.c_void_p()
    rc = L.lib().ns_create(ctypes.byref(desc), ctypes.byref(prm), ctypes.byref(h))
    return rc, h


def test_zeroed_params_select_multigrid(gpu):
    L = gpu._lib
    n = 256
    prm = L.NsParams()              # ctypes zero-initialises every field
    prm.dt, prm.re, prm.nranks = 1.0 / (8 * n), 100.0, 1
    assert prm.poisson == L.NS_POISSON_MG == 0
    rc, h = _create(L, n, prm)
    assert rc == 0, L.lib().ns_last_error()
    try:
        for _ in range(3):
            st = L.NsStats()
            assert L.lib().ns_step(h, ctypes.byref(st)) == 0, L.lib().ns_last_error()
            # V-cycles (a handful), not the O(n) RB-SOR sweeps of ABI 3's zero value
            assert 1 <= st.it_phi <= 12
            # (the direct solve checks its residual on the first solve and every 16th: res_phi = -1 between)
            assert (st.phi_checked == 1 and 0 <= st.res_phi <= 1e-8) or (st.phi_checked == 0 and st.res_phi == -1.0)
    finally:
        L.lib().ns_destroy(h)


def test_retired_poisson_value_is_rejected(gpu):
    L = gpu._lib
    prm = L.NsParams()
    prm.dt, prm.re, prm.nranks, prm.poisson = 1.0 / 512, 100.0, 1, 2
    rc, h = _create(L, 64, prm)
    assert rc == L.NS_EINVAL and not h.value
    assert b"unknown Poisson solver 2" in L.lib().ns_last_error()
