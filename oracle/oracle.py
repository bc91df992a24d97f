"""ctypes wrapper of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / timed CPU baseline (see ns_oracle.h for
provenance and how the oracle is pinned)."""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

_D = ctypes.POINTER(ctypes.c_double)
_I = ctypes.POINTER(ctypes.c_int)
_P = ctypes.c_void_p
_SIG = {
    "og_last_error": (ctypes.c_char_p, []),
    "og_set_threads": (None, [ctypes.c_int]),
    "og_get_threads": (ctypes.c_int, []),
    "og_grid_polygon": (_P, [ctypes.c_int, _D, _D, ctypes.c_int, _D, ctypes.c_int, _D, _I, _D]),
    "og_grid_free": (None, [_P]),
    "og_grid_N": (ctypes.c_int, [_P]),
    "og_grid_nx": (ctypes.c_int, [_P]),
    "og_grid_ny": (ctypes.c_int, [_P]),
    "og_grid_info": (None, [_P, _D, _D, _I, _I, _D, _D]),
    "og_grad_phi": (None, [_P, _D, _D, _D]),
    "og_rhs_velocity": (None, [_P, ctypes.c_double, ctypes.c_double, _D, _D, _D, _D, _D, _D, _D, _D]),
    "og_divergence": (None, [_P, ctypes.c_double, _D, _D, _D]),
    "og_correct": (None, [_P, ctypes.c_double, _D, _D, _D, _D, _D, _D, _D]),
    "og_apply_poisson": (None, [_P, _D, _D]),
    "og_apply_helmholtz": (None, [_P, ctypes.c_double, _D, _D]),
    "og_pressure": (None, [_P, ctypes.c_double, _D, _D]),
    "og_poisson_jacobi_sweep": (ctypes.c_double, [_P, _D, _D, _D, ctypes.c_double, ctypes.c_double]),
    "og_poisson_rbsor_sweep": (ctypes.c_double, [_P, _D, _D, ctypes.c_double, ctypes.c_double]),
    "og_helmholtz_rbsor_sweep": (ctypes.c_double, [_P, ctypes.c_double, _D, _D, _D, _D, ctypes.c_double]),
    "og_solve_helmholtz": (ctypes.c_int, [_P, ctypes.c_double, _D, _D, ctypes.c_double, ctypes.c_int]),
    "og_solve_poisson": (ctypes.c_int, [_P, _D, _D, ctypes.c_double, ctypes.c_int]),
    "og_mg_restrict": (None, [ctypes.c_int, ctypes.c_int, _D, _D, _D, _D, ctypes.c_double, _D]),
    "og_mg_prolong": (None, [ctypes.c_int, ctypes.c_int, _D, _D]),
    "og_mg_set_direct": (None, [ctypes.c_long]),
    "og_mg_solve": (ctypes.c_int, [_P, _D, _D, ctypes.c_double, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "og_mg_solve_w": (ctypes.c_int, [_P, _D, _D, ctypes.c_double, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_double]),
    "og_fps_ok": (ctypes.c_int, [_P]),
    "og_fps_solve": (ctypes.c_int, [_P, _D, _D]),
    "og_solver_set_algorithm": (None, [_P, ctypes.c_int, ctypes.c_double, ctypes.c_double]),
    "og_solver_set_band": (None, [_P, ctypes.c_int, ctypes.c_int]),
    "og_helm_band": (ctypes.c_int, [_P, ctypes.c_double, _D, _D, _D, _D, ctypes.c_double, ctypes.c_int, ctypes.c_int]),
    "og_solver_new": (_P, [_P, ctypes.c_double, ctypes.c_double, ctypes.c_double]),
    "og_solver_free": (None, [_P]),
    "og_solver_step": (ctypes.c_int, [_P, _D, _I]),
    "og_solver_get": (None, [_P, _D, _D, _D, _D, _D, _D, _D]),
    "og_solver_set": (None, [_P, _D, _D, _D, _D, _D, _D, _D]),
}
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run `make -C oracle`")
        L = ctypes.CDLL(LIB_PATH)
        for k, (r, a) in _SIG.items():
            f = getattr(L, k)
            f.restype, f.argtypes = r, a
        _lib = L
    return _lib


def set_direct_cells(n: int) -> None:
    """The multigrid's exact coarsest-level solve threshold (the GPU's NSGPU_DIRECT_CELLS; default
    128^2, 0 = off) -- set both sides alike when a test changes it."""
    lib().og_mg_set_direct(int(n))


def set_threads(n: int) -> None:
    """OpenMP threads of the restatement's per-cell loops (default 1)."""
    lib().og_set_threads(int(n))


def _d(a):
    return a.ctypes.data_as(_D) if a is not None else None


def _f(a):
    return np.ascontiguousarray(a, dtype=np.float64)


class OGrid:
    """Grid built by the oracle's restatement of Grid.cpp (polygon -> cells, ids, tags)."""

    def __init__(self, vertices, xspec, yspec, bc):
        vx = _f([v[0] for v in vertices]); vy = _f([v[1] for v in vertices])
        xs = _f(np.asarray(xspec, dtype=np.float64).ravel()); ys = _f(np.asarray(yspec, dtype=np.float64).ravel())
        bt = np.ascontiguousarray([int(t) for t, _ in bc], dtype=np.intc)
        bi = _f([float(i) for _, i in bc])
        h = lib().og_grid_polygon(len(vertices), _d(vx), _d(vy), xs.size // 4, _d(xs), ys.size // 4, _d(ys),
                                  bt.ctypes.data_as(_I), _d(bi))
        if not h:
            raise ValueError(lib().og_last_error().decode())
        self.h = h
        self.N = lib().og_grid_N(h)
        self.nx = lib().og_grid_nx(h)
        self.ny = lib().og_grid_ny(h)
        self.hx = np.empty(self.nx); self.hy = np.empty(self.ny)
        self.id = np.empty(self.nx * self.ny, dtype=np.intc)
        self.tag = np.empty(self.nx * self.ny * 4, dtype=np.intc)
        self.xc = np.empty(self.N); self.yc = np.empty(self.N)
        lib().og_grid_info(h, _d(self.hx), _d(self.hy), self.id.ctypes.data_as(_I), self.tag.ctypes.data_as(_I),
                           _d(self.xc), _d(self.yc))

    @classmethod
    def rectangle(cls, nx, ny, lx=1.0, ly=1.0, bc=None, xratio=-1, yratio=-1):
        if bc is None:
            bc = [(2, 0.0), (2, 1.0), (2, 0.0), (2, 0.0)]
        return cls([(0, 0), (0, ly), (lx, ly), (lx, 0)], [[0, lx, nx, xratio]], [[0, ly, ny, yratio]], bc)

    def __del__(self):
        try:
            lib().og_grid_free(self.h)
        except Exception:
            pass

    def z(self):
        return np.zeros(self.N)

    # ---- kernels
    def grad_phi(self, phi):
        gx, gy = self.z(), self.z()
        lib().og_grad_phi(self.h, _d(_f(phi)), _d(gx), _d(gy))
        return gx, gy

    def rhs_velocity(self, dt, re, u, v, gx, gy, cu, cv):
        cu, cv = _f(cu).copy(), _f(cv).copy()
        ru, rv = self.z(), self.z()
        lib().og_rhs_velocity(self.h, dt, re, _d(_f(u)), _d(_f(v)), _d(_f(gx)), _d(_f(gy)), _d(cu), _d(cv),
                              _d(ru), _d(rv))
        return ru, rv, cu, cv

    def divergence(self, dt, us, vs):
        out = self.z()
        lib().og_divergence(self.h, dt, _d(_f(us)), _d(_f(vs)), _d(out))
        return out

    def correct(self, dt, us, vs, phi):
        u, v, gx, gy = self.z(), self.z(), self.z(), self.z()
        lib().og_correct(self.h, dt, _d(_f(us)), _d(_f(vs)), _d(_f(phi)), _d(u), _d(v), _d(gx), _d(gy))
        return u, v, gx, gy

    def apply_poisson(self, phi):
        out = self.z()
        lib().og_apply_poisson(self.h, _d(_f(phi)), _d(out))
        return out

    def apply_helmholtz(self, alpha, q):
        out = self.z()
        lib().og_apply_helmholtz(self.h, alpha, _d(_f(q)), _d(out))
        return out

    def pressure(self, alpha, phi):
        out = self.z()
        lib().og_pressure(self.h, alpha, _d(_f(phi)), _d(out))
        return out

    def jacobi_sweep(self, phi, b, shift, omega):
        out = self.z()
        r2 = lib().og_poisson_jacobi_sweep(self.h, _d(_f(phi)), _d(out), _d(_f(b)), shift, omega)
        return out, r2

    def rbsor_sweep(self, phi, b, shift, omega):
        p = _f(phi).copy()
        r2 = lib().og_poisson_rbsor_sweep(self.h, _d(p), _d(_f(b)), shift, omega)
        return p, r2

    def helm_sweep(self, alpha, u, v, ru, rv, omega=1.0):
        u, v = _f(u).copy(), _f(v).copy()
        r2 = lib().og_helmholtz_rbsor_sweep(self.h, alpha, _d(u), _d(v), _d(_f(ru)), _d(_f(rv)), omega)
        return u, v, r2

    def band_width(self):
        """The GPU's default wall-band width: 1/32 of the shorter side, at least 32 cells."""
        return max(32, min(self.nx, self.ny) // 32)

    def helm_band(self, alpha, u, v, ru, rv, omega=1.0, width=None, sweeps=6):
        """k_helm_band restated: RB-SOR sweeps of u, v on the cells within `width` of a wall
        (None: the GPU's default, band_width())."""
        width = self.band_width() if width is None else width
        u, v = _f(u).copy(), _f(v).copy()
        if lib().og_helm_band(self.h, alpha, _d(u), _d(v), _d(_f(ru)), _d(_f(rv)), omega, width, sweeps) != 0:
            raise ValueError(lib().og_last_error().decode())
        return u, v

    def solve_helmholtz(self, alpha, rhs, x0=None, rtol=1e-13, maxit=100000):
        x = self.z() if x0 is None else _f(x0).copy()
        it = lib().og_solve_helmholtz(self.h, alpha, _d(_f(rhs)), _d(x), rtol, maxit)
        return x, it

    def mg_restrict(self, phi, b, shift):
        bc = np.zeros((self.nx // 2) * (self.ny // 2))
        lib().og_mg_restrict(self.nx, self.ny, _d(self.hx), _d(self.hy), _d(_f(phi)), _d(_f(b)), shift, _d(bc))
        return bc

    def mg_prolong(self, phi, ec):
        p = _f(phi).copy()
        lib().og_mg_prolong(self.nx, self.ny, _d(_f(ec)), _d(p))
        return p

    def mg_solve(self, rhs, x0=None, rtol=1e-10, pre=2, post=2, maxcycles=1000, omega=1.0):
        b = _f(rhs).copy()
        x = self.z() if x0 is None else _f(x0).copy()
        cyc = lib().og_mg_solve_w(self.h, _d(b), _d(x), rtol, pre, post, maxcycles, omega)
        if cyc < 0:
            raise ValueError(lib().og_last_error().decode())
        return x, cyc

    def fps_ok(self):
        """The GPU's direct Poisson solve applies (a uniform rectangle with zero-flux phi faces,
        ny = 2^p in [16, 16384]): the GPU's default Poisson solve there (NSGPU_FPS)."""
        return bool(lib().og_fps_ok(self.h))

    def fps_solve(self, rhs):
        """The direct solve (DCT along y, Thomas along x, mode 0 pinned) of L x = rhs - mean."""
        b = _f(rhs).copy()
        x = self.z()
        if lib().og_fps_solve(self.h, _d(b), _d(x)) < 0:
            raise ValueError(lib().og_last_error().decode())
        return x

    def solve_poisson(self, rhs, x0=None, rtol=1e-13, maxit=100000):
        b = _f(rhs).copy()
        x = self.z() if x0 is None else _f(x0).copy()
        it = lib().og_solve_poisson(self.h, _d(b), _d(x), rtol, maxit)
        return x, it


class OSolver:
    """FluidSolver::Solve restated (converged linear solves)."""

    def __init__(self, grid: OGrid, dt, re, rtol=1e-13):
        self.g = grid
        self.h = lib().og_solver_new(grid.h, dt, re, rtol)
        self.dt, self.re = dt, re

    def __del__(self):
        try:
            lib().og_solver_free(self.h)
        except Exception:
            pass

    def use_gpu_algorithm(self, omega_v, omega_mg=1.1, band=(None, 6), fps=True):
        """RB-SOR Helmholtz (after `band` = (width, sweeps) RB-SOR sweeps on the cells within
        `width` of a wall: k_helm_band; width None = the GPU's default, band=None = no band step)
        + the Poisson solve of the GPU path: the direct solve where it applies (fps, the GPU's
        NSGPU_FPS default), multigrid otherwise (CPU baseline)."""
        lib().og_solver_set_algorithm(self.h, 2 if fps else 1, omega_v, omega_mg)
        w, k = band if band else (0, 0)
        if band and w is None:
            w = self.g.band_width()
        lib().og_solver_set_band(self.h, w, k)

    def step(self):
        mm = np.zeros(4)
        its = np.zeros(3, dtype=np.intc)
        lib().og_solver_step(self.h, _d(mm), its.ctypes.data_as(_I))
        return mm, its

    def get(self):
        a = [self.g.z() for _ in range(7)]
        lib().og_solver_get(self.h, *[_d(x) for x in a])
        return dict(zip(["u", "v", "phi", "cu", "cv", "gx", "gy"], a))

    def set(self, u=None, v=None, phi=None, cu=None, cv=None, gx=None, gy=None):
        args = [None if x is None else _f(x) for x in (u, v, phi, cu, cv, gx, gy)]
        lib().og_solver_set(self.h, *[_d(x) for x in args])
