"""Which closure of the outflow side should the Poisson preconditioner's multigrid relax?

Builds, on a uniform nx x ny channel (walls S/N and W, the reference's NEUMANN outflow on E:
phi ghost 2.5 phi_c - 2 phi_1 + 0.5 phi_2, FluidSolver.cpp:98-101), the true Poisson matrix
and three closures of the same stencil -- wall (ghost phi_c), linear extrapolation (2 phi_c -
phi_1) and partial ones (phi_c + theta (phi_c - phi_1)) -- and counts the BiCGStab iterations
to rtol 1e-8 with an EXACT solve of each closure as the preconditioner (null spaces handled
by projection).  Result (the MG preconditioner approximates these):
  64x32:   wall 16, linear 5, theta 0.9: 7, 0.75: 10, 0.5: 12
  256x128: wall 35, linear 5, theta 0.9: 12, 0.75: 19, 0.5: 24
The exact-solve advantage did NOT carry over to the GPU's one-V-cycle preconditioner: with
the closure in every level's tables (and in the LDS coarse V-cycle) the 4096x1024 channel
needed 42 (wall), 50 (0.5), 77 (0.75), 82 (0.9), 58 (1.0) BiCGStab iterations per step --
the rediscretised closure is a poor coarse-grid approximation (theta = 1 on a uniform grid
even decouples the outflow column in x).  Reverted; DESIGN.md section 9.
  python tools/outflow_pc_proto.py     (CPU, scipy; ~1 min)
"""
import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla


def op(nx, ny, closure):
    N = nx * ny
    idx = lambda i, j: i * ny + j
    A = sp.lil_matrix((N, N))
    for i in range(nx):
        for j in range(ny):
            r, d = idx(i, j), 0.0
            for di, dj in ((-1, 0), (1, 0), (0, -1), (0, 1)):
                ii, jj = i + di, j + dj
                if 0 <= ii < nx and 0 <= jj < ny:
                    A[r, idx(ii, jj)] += 1
                    d -= 1
                elif di == 1:   # the E outflow face: (ghost - phi_c) / h^2
                    if closure == "true":
                        A[r, r] += 1.5; A[r, idx(i - 1, j)] += -2; A[r, idx(i - 2, j)] += 0.5
                    elif closure != "wall":
                        th = 1.0 if closure == "linear" else float(closure)
                        A[r, r] += th; A[r, idx(i - 1, j)] += -th
            A[r, r] += d
    return A.tocsr()


def left_null(A, k):
    AT = A.T.tolil()
    AT[k, :] = 0
    AT[k, k] = 1.0
    e = np.zeros(A.shape[0])
    e[k] = 1.0
    return spla.spsolve(AT.tocsc(), e)


for nx, ny in ((64, 32), (256, 128)):
    A = op(nx, ny, "true")
    k = (nx - 1) * ny
    w = left_null(A, k)
    b = np.random.default_rng(0).standard_normal(nx * ny)
    b -= w * (w @ b) / (w @ w)
    out = []
    for cl in ("wall", "linear", "0.9", "0.75", "0.5"):
        M = op(nx, ny, cl)
        wc = left_null(M, k if cl != "wall" else 0)
        Mp = M.tolil()
        Mp[k, :] = 0
        Mp[k, k] = 1.0
        lu = spla.splu(Mp.tocsc())

        def apply(r, lu=lu, wc=wc):
            z = lu.solve(r - wc * (wc @ r) / (wc @ wc))
            return z - z.mean()

        its = [0]
        x, info = spla.bicgstab(A, b, M=spla.LinearOperator(A.shape, matvec=apply), rtol=1e-8, maxiter=3000,
                                callback=lambda xk: its.__setitem__(0, its[0] + 1))
        out.append(f"{cl}: {its[0]}")
    print(f"{nx}x{ny}", ", ".join(out), flush=True)
