"""navierstokessolver_amd -- MI355X (gfx950) implementation of the
shivams15/navierstokessolver hot path (FluidSolver::Solve's advect/diffuse/project
step and its pressure-Poisson solve) behind a C-ABI (include/nsgpu.h).

The compute path is libnsgpu.so (hand-written HIP kernels + RCCL halos); this
package is the ctypes plumbing used by tests/ and bench.py.  The drop-in for the
reference's own driver is the C++ Grid / FluidSolver in host/.
"""
from . import _lib
from ._lib import (NS_ARR_CU, NS_ARR_CV, NS_ARR_PHI, NS_ARR_RPHI, NS_ARR_RU, NS_ARR_RV, NS_ARR_TMP,
                   NS_ARR_U, NS_ARR_V, NS_BC_INLET_UNI, NS_BC_NEUMANN, NS_BC_WALL, NS_K_CORRECT, NS_K_DIV,
                   NS_K_HELM_BAND, NS_K_HELM_SOLVE, NS_K_HELMHOLTZ, NS_K_POIS_SOLVE, NS_K_POISSON, NS_K_POISSON32, NS_K_RESIDUAL, NS_K_RHS,
                   NS_POISSON_JACOBI, NS_POISSON_MG, NS_POISSON_RBSOR, NsError, slab_range)
from .cavity import cavity, cavity_dt, polygon, rectangle
from .solver import Edge, GpuSolver, GridSpec

__all__ = [n for n in dir() if not n.startswith("_")]
