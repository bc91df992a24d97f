"""Python handle over one ns_solver (libnsgpu.so).  Plumbing for tests and bench.py;
the reference-compatible host API is the C++ Grid / FluidSolver in host/."""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L


@dataclass
class Edge:
    """One polygon edge (Edge, /root/reference/SRC/Grid.h:20-26)."""
    nx: int
    ny: int
    type: int = L.NS_BC_WALL
    info: float = 0.0


@dataclass
class GridSpec:
    """Geometry handed to ns_create: spacings plus edges.  A rectangle leaves cell_id /
    face_edge None; any other polygon (cavity.polygon) carries the bounding box's
    compact ids (-1 outside; Grid.cpp:149-162) and per-cell boundary-edge tags (W,E,S,N;
    Cell::edges, Grid.h:33)."""
    hx: np.ndarray
    hy: np.ndarray
    edges: list = field(default_factory=list)
    cell_id: np.ndarray | None = None
    face_edge: np.ndarray | None = None

    @property
    def mask(self):
        """nx x ny booleans: the cells inside the domain (all of them for a rectangle)."""
        if self.cell_id is None:
            return np.ones((self.nx, self.ny), dtype=bool)
        return np.asarray(self.cell_id).reshape(self.nx, self.ny) >= 0

    @property
    def nx(self):
        return len(self.hx)

    @property
    def ny(self):
        return len(self.hy)


def _dptr(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


class GpuSolver:
    """One x-slab (the whole grid when nranks == 1) resident on one MI355X."""

    def __init__(self, grid: GridSpec, dt: float, re: float, *, poisson=L.NS_POISSON_MG, rtol=1e-8,
                 max_iters=0, omega=0.0, omega_v=0.0, check_every=0, device=-1, timing=False,
                 rank=0, nranks=1, nccl_id: bytes | None = None, mg_pre=0, mg_post=0, mg_coarse_iters=0,
                 host_transport=None, mg_omega=0.0):
        self.grid = grid
        self.hx = np.ascontiguousarray(grid.hx, dtype=np.float64)
        self.hy = np.ascontiguousarray(grid.hy, dtype=np.float64)
        self._edges = (L.NsEdge * len(grid.edges))(*[L.NsEdge(e.nx, e.ny, e.type, e.info) for e in grid.edges])
        ip = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        self._cid = self._ftag = None
        if grid.cell_id is not None:
            self._cid = np.ascontiguousarray(grid.cell_id, dtype=np.int32)
            self._ftag = np.ascontiguousarray(grid.face_edge, dtype=np.int32)
            assert self._cid.size == self.hx.size * self.hy.size and self._ftag.size == 4 * self._cid.size
        desc = L.NsGridDesc(self.hx.size, self.hy.size, _dptr(self.hx), _dptr(self.hy), len(grid.edges),
                            self._edges, ip(self._cid) if self._cid is not None else None,
                            ip(self._ftag) if self._ftag is not None else None)
        self._nccl = ctypes.create_string_buffer(nccl_id, len(nccl_id)) if nccl_id else None
        prm = L.NsParams(dt, re, poisson, rtol, max_iters, omega, omega_v, check_every, device,
                         1 if timing else 0, rank, nranks,
                         ctypes.cast(self._nccl, ctypes.c_void_p) if self._nccl is not None else None,
                         mg_pre, mg_post, mg_coarse_iters,
                         ctypes.pointer(host_transport.struct) if host_transport is not None else None,
                         mg_omega)
        self._transport = host_transport  # keep the callbacks alive
        h = ctypes.c_void_p()
        L.check(L.lib().ns_create(ctypes.byref(desc), ctypes.byref(prm), ctypes.byref(h)))
        self._h = h
        self.dt, self.re = dt, re
        self.rank, self.nranks = rank, nranks
        self.i0, self.i1 = L.slab_range(self.hx.size, nranks, rank)
        # the Helmholtz SOR weight libnsgpu.so derives (ns_create): 2 / (1 + sqrt(1 - rho^2))
        if omega_v > 0:
            self.omega_v = omega_v
        else:
            t = dt / re * (1 / self.hx.min() ** 2 + 1 / self.hy.min() ** 2)
            rho = t / (1 + t)
            self.omega_v = 2 / (1 + (1 - rho * rho) ** 0.5)
        self.shape = (self.i1 - self.i0, self.hy.size)
        # the multigrid smoother's over-relaxation (ns_create: 1.1 unless given; NSGPU_MG_OMEGA wins)
        self.mg_omega = float(os.environ.get("NSGPU_MG_OMEGA", mg_omega if mg_omega > 0 else 1.1))

    # ---- lifecycle
    def close(self):
        if getattr(self, "_h", None):
            L.lib().ns_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- stepping
    def step(self) -> dict:
        st = L.NsStats()
        L.check(L.lib().ns_step(self._h, ctypes.byref(st)))
        return st.as_dict()

    def step_async(self) -> dict:
        """ns_step_async: one step without the closing host sync; umin..vmax are the previous
        step_async's monitor values (NaN on the first), monitor() returns the latest."""
        st = L.NsStats()
        L.check(L.lib().ns_step_async(self._h, ctypes.byref(st)))
        return st.as_dict()

    def monitor(self) -> tuple:
        mm = np.empty(4, dtype=np.float64)
        L.check(L.lib().ns_monitor(self._h, _dptr(mm)))
        return tuple(float(x) for x in mm)

    # ---- state
    def get(self, which: int) -> np.ndarray:
        out = np.empty(self.shape, dtype=np.float64)
        L.check(L.lib().ns_get_array(self._h, which, _dptr(out)))
        return out

    def set(self, which: int, a) -> None:
        a = np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(self.shape))
        L.check(L.lib().ns_set_array(self._h, which, _dptr(a)))

    def fields(self):
        """u, v, phi as the slab's nx_local x ny bounding-box planes (ns_get_array)."""
        return self.get(L.NS_ARR_U), self.get(L.NS_ARR_V), self.get(L.NS_ARR_PHI)

    def local_cells(self) -> tuple:
        """(first compact id, count) of this slab's in-domain cells (ns_local_cells)."""
        a, n = ctypes.c_int64(), ctypes.c_int64()
        L.check(L.lib().ns_local_cells(self._h, ctypes.byref(a), ctypes.byref(n)))
        return a.value, n.value

    def fields_compact(self):
        """u, v, phi in the reference's compact Vec order (ns_get_fields; Grid.cpp:149-162)."""
        n = self.local_cells()[1]
        u, v, p = (np.empty(n) for _ in range(3))
        L.check(L.lib().ns_get_fields(self._h, _dptr(u), _dptr(v), _dptr(p)))
        return u, v, p

    def set_fields_compact(self, u=None, v=None, phi=None, cu0=None, cv0=None) -> None:
        """ns_set_fields: any of u, v, phi, convectiveDer_u0 / _v0 in compact Vec order."""
        n = self.local_cells()[1]
        keep = [None if a is None else np.ascontiguousarray(np.asarray(a, dtype=np.float64).ravel())
                for a in (u, v, phi, cu0, cv0)]
        for a in keep:
            if a is not None and a.size != n:
                raise ValueError(f"compact field of {a.size} values; this slab holds {n} cells")
        L.check(L.lib().ns_set_fields(self._h, *[None if a is None else _dptr(a) for a in keep]))

    def kernel(self, which: int, iters: int = 1) -> np.ndarray:
        out = np.zeros(8, dtype=np.float64)
        L.check(L.lib().ns_kernel(self._h, which, iters, _dptr(out)))
        return out

    def mg_restrict(self) -> np.ndarray:
        out = np.zeros((self.shape[0] // 2, self.shape[1] // 2))
        L.check(L.lib().ns_mg_transfer(self._h, 0, _dptr(out)))
        return out

    def mg_prolong(self, coarse) -> None:
        c = np.ascontiguousarray(np.asarray(coarse, dtype=np.float64).reshape(self.shape[0] // 2, self.shape[1] // 2))
        L.check(L.lib().ns_mg_transfer(self._h, 1, _dptr(c)))

    def set_timing(self, on: bool) -> None:
        L.check(L.lib().ns_set_timing(self._h, 1 if on else 0))

    def fill_random(self, seed: int = 0x5EED) -> None:
        L.check(L.lib().ns_fill_random(self._h, seed))

    def time_poisson(self, warmup: int, iters: int):
        out = np.zeros(3, dtype=np.float64)
        L.check(L.lib().ns_time_poisson(self._h, warmup, iters, _dptr(out)))
        return {"avg_ms": out[0], "total_ms": out[1], "span_ms": out[2]}

    def time_poisson_fp32(self, warmup: int, iters: int):
        """Jacobi sweeps on fp32 copies of phi, rhs_phi (configs[4]); also the fp64-summed
        residual^2 of the last sweep's input."""
        out = np.zeros(4, dtype=np.float64)
        L.check(L.lib().ns_time_poisson_fp32(self._h, warmup, iters, _dptr(out)))
        return {"avg_ms": out[0], "total_ms": out[1], "span_ms": out[2], "res2": out[3]}
