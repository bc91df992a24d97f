"""ctypes binding of libnsgpu.so (include/nsgpu.h).

The shared library is built in-tree (``python -c "import __graft_entry__ as g; g.build()"``
or ``make -C navierstokessolver_amd/csrc``).  There is deliberately no CPU fallback:
if the library or the GPU is missing, every call fails loudly.
"""
from __future__ import annotations

import ctypes
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NSGPU_LIB", os.path.join(HERE, "libnsgpu.so"))
HEADER = os.path.join(os.path.dirname(HERE), "include", "nsgpu.h")

# ---- constants mirrored from include/nsgpu.h (checked by tests/test_abi.py) ----
NSGPU_ABI_VERSION = 9   # the struct layouts / enum values below; lib() refuses a library of another ABI
NS_OK, NS_EINVAL, NS_EHIP, NS_ERCCL, NS_ENOMEM, NS_EDIVERGE = 0, -1, -2, -3, -4, -5
NS_BC_INLET_UNI, NS_BC_INLET_PARABOLIC, NS_BC_WALL, NS_BC_PRESSURE, NS_BC_NEUMANN = 0, 1, 2, 3, 4
NS_POISSON_MG, NS_POISSON_JACOBI, NS_POISSON_RBSOR = 0, 1, 3   # ABI 4: zeroed params select MG
(NS_ARR_U, NS_ARR_V, NS_ARR_PHI, NS_ARR_CU, NS_ARR_CV, NS_ARR_RU, NS_ARR_RV, NS_ARR_RPHI,
 NS_ARR_TMP, NS_ARR_TMPU, NS_ARR_TMPV) = range(11)
NS_NUM_ARR = 11
(NS_K_RHS, NS_K_HELMHOLTZ, NS_K_DIV, NS_K_POISSON, NS_K_CORRECT, NS_K_HELM_SOLVE,
 NS_K_POIS_SOLVE, NS_K_RESIDUAL, NS_K_POISSON32, NS_K_HELM_BAND) = range(1, 11)


class NsEdge(ctypes.Structure):
    _fields_ = [("nx", ctypes.c_int32), ("ny", ctypes.c_int32), ("type", ctypes.c_int32),
                ("info", ctypes.c_double)]


class NsGridDesc(ctypes.Structure):
    _fields_ = [("nx", ctypes.c_int32), ("ny", ctypes.c_int32),
                ("hx", ctypes.POINTER(ctypes.c_double)), ("hy", ctypes.POINTER(ctypes.c_double)),
                ("n_edges", ctypes.c_int32), ("edges", ctypes.POINTER(NsEdge)),
                ("cell_id", ctypes.POINTER(ctypes.c_int32)), ("face_edge", ctypes.POINTER(ctypes.c_int32))]


EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                               ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                               ctypes.POINTER(ctypes.c_double), ctypes.c_int64)
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_int32,
                                ctypes.c_int32)


class NsHostTransport(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("exchange", EXCHANGE_FN), ("allreduce", ALLREDUCE_FN)]


class NsParams(ctypes.Structure):
    _fields_ = [("dt", ctypes.c_double), ("re", ctypes.c_double), ("poisson", ctypes.c_int32),
                ("rtol", ctypes.c_double), ("max_iters", ctypes.c_int32), ("omega", ctypes.c_double),
                ("omega_v", ctypes.c_double), ("check_every", ctypes.c_int32),
                ("device", ctypes.c_int32), ("timing", ctypes.c_int32),
                ("rank", ctypes.c_int32), ("nranks", ctypes.c_int32), ("nccl_id", ctypes.c_void_p),
                ("mg_pre", ctypes.c_int32), ("mg_post", ctypes.c_int32), ("mg_coarse_iters", ctypes.c_int32),
                ("host_transport", ctypes.POINTER(NsHostTransport)), ("mg_omega", ctypes.c_double)]


class NsStats(ctypes.Structure):
    _fields_ = [("umin", ctypes.c_double), ("umax", ctypes.c_double), ("vmin", ctypes.c_double),
                ("vmax", ctypes.c_double), ("it_u", ctypes.c_int32), ("it_v", ctypes.c_int32),
                ("it_phi", ctypes.c_int32), ("res_u", ctypes.c_double), ("res_v", ctypes.c_double),
                ("res_phi", ctypes.c_double), ("t_poisson_kernel_ms", ctypes.c_double),
                ("n_poisson_kernels", ctypes.c_int32), ("n_checks", ctypes.c_int32),
                ("t_restrict_kernel_ms", ctypes.c_double), ("n_restrict_kernels", ctypes.c_int32),
                ("t_helm_kernel_ms", ctypes.c_double), ("n_helm_kernels", ctypes.c_int32),
                ("n_exchanges", ctypes.c_int32), ("n_allreduces", ctypes.c_int32),
                ("x_link_bytes", ctypes.c_double), ("t_cycle_kernel_ms", ctypes.c_double),
                ("n_cycle_kernels", ctypes.c_int32), ("t_guess_kernel_ms", ctypes.c_double),
                ("n_guess_kernels", ctypes.c_int32), ("t_rhs_kernel_ms", ctypes.c_double),
                ("n_rhs_kernels", ctypes.c_int32), ("t_fps_dct_ms", ctypes.c_double), ("t_fps_tri_ms", ctypes.c_double),
                ("t_fps_idct_ms", ctypes.c_double), ("n_fps_solves", ctypes.c_int32),
                ("phi_checked", ctypes.c_int32), ("t_k5_kernel_ms", ctypes.c_double),
                ("n_k5_kernels", ctypes.c_int32), ("t_band_kernel_ms", ctypes.c_double),
                ("n_band_kernels", ctypes.c_int32), ("k5_deferred", ctypes.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_P = ctypes.c_void_p
_D = ctypes.POINTER(ctypes.c_double)
SIGNATURES = {
    "ns_create": (ctypes.c_int, [ctypes.POINTER(NsGridDesc), ctypes.POINTER(NsParams), ctypes.POINTER(_P)]),
    "ns_destroy": (None, [_P]),
    "ns_step": (ctypes.c_int, [_P, ctypes.POINTER(NsStats)]),
    "ns_step_async": (ctypes.c_int, [_P, ctypes.POINTER(NsStats)]),
    "ns_monitor": (ctypes.c_int, [_P, _D]),
    "ns_get_fields": (ctypes.c_int, [_P, _D, _D, _D]),
    "ns_set_fields": (ctypes.c_int, [_P, _D, _D, _D, _D, _D]),
    "ns_local_cells": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    "ns_get_array": (ctypes.c_int, [_P, ctypes.c_int, _D]),
    "ns_set_array": (ctypes.c_int, [_P, ctypes.c_int, _D]),
    "ns_kernel": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, _D]),
    "ns_fill_random": (ctypes.c_int, [_P, ctypes.c_uint64]),
    "ns_mg_transfer": (ctypes.c_int, [_P, ctypes.c_int, _D]),
    "ns_time_poisson": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, _D]),
    "ns_time_poisson_fp32": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, _D]),
    "ns_set_timing": (ctypes.c_int, [_P, ctypes.c_int]),
    "ns_slab_range": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                     ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]),
    "ns_nccl_id_size": (ctypes.c_int, []),
    "ns_nccl_get_id": (ctypes.c_int, [_P]),
    "ns_device_bytes": (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int32]),
    "ns_abi_version": (ctypes.c_int, []),
    "ns_last_error": (ctypes.c_char_p, []),
}

_lib = None


class NsError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"libnsgpu error {code}: {msg}")
        self.code = code


def lib():
    """Load libnsgpu.so once; raise (never fall back) if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
                              "(there is no CPU fallback for the product path)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name, None)   # (an older library under NSGPU_LIB: a missing entry point
            if fn is None:                #  raises when called; tests/test_abi.py checks the export list)
                continue
            fn.restype = res
            fn.argtypes = args
        # these bindings mirror one ABI's ns_params / ns_stats layouts and enum values: a library of
        # another ABI would read them wrongly (or write past a shorter ns_stats) -- refuse it
        abi = L.ns_abi_version()
        if abi != NSGPU_ABI_VERSION:
            raise ImportError(f"{LIB_PATH} has ABI {abi}; these bindings expect ABI {NSGPU_ABI_VERSION} "
                              "(rebuild with __graft_entry__.build())")
        _lib = L
    return _lib


def check(rc):
    if rc != 0:
        raise NsError(rc, lib().ns_last_error().decode(errors="replace"))
    return rc


def header_functions(path=HEADER):
    """Names of every function prototype declared in include/nsgpu.h."""
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\*?\s*([a-z_][a-z0-9_]*)\s*\(", txt, flags=re.M)
    return sorted(set(n for n in names if n.startswith("ns_")))


def slab_range(nx, nranks, rank):
    a, b = ctypes.c_int32(), ctypes.c_int32()
    check(lib().ns_slab_range(nx, nranks, rank, ctypes.byref(a), ctypes.byref(b)))
    return a.value, b.value
