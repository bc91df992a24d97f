"""How should the Poisson preconditioner treat a NEUMANN outflow side?  

On a uniform nx x ny channel (h = 1; walls W, S, N; the reference's outflow on E: phi ghost
2.5 phi_c - 2 phi_1 + 0.5 phi_2, FluidSolver.cpp:98-101) this builds the true Poisson matrix
and counts BiCGStab iterations (rtol 1e-8, mean-projected system, random rhs) for:

  wall        one V-cycle of the wall-closure multigrid (round 1)
  line/exact  the line-closure preconditioner with exact solves: the outflow row's stencil is
              0.5 phi_xx + phi_yy, so its value is ~ Ly^-1 r_E (a 1-D Neumann solve along the
              side); that line solution becomes face-Dirichlet data g of the side, and
              z = D^-1 (r - 2 g / h^2 e_E) with D the Laplacian closed there by a face-Dirichlet
              condition (weight 2/h^2 toward the face)
  line/v0     the same with D^-1 replaced by one V(2,2)-cycle started from z = 0
  line/vext   ... started from z0 = g extended constantly along x.  D z0 is O(r), so the cycle
              works on an O(r) residual instead of the O(ny^2 r) Dirichlet data, and its error
              no longer grows with ny -- what the GPU does (mg_precond, k_line_solve,
              k_line_extend; prolongation odd at the face-Dirichlet side)

Result:
  64x32:   wall 18, line/exact 6, line/v0 9,  line/vext 7
  256x64:  wall 24, line/exact 6, line/v0 10, line/vext 8
  256x128: wall 36, line/exact 7, line/v0 16, line/vext 8
On the MI355X (tools/outflow_pc_diag.py, channel with square cells, per step from rest):
line 6-9 iterations at 1024x256 .. 4096x1024, wall 30-68.
  python tools/outflow_pc_proto.py     (CPU, numpy + scipy; ~1 min)
"""
import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla


def true_op(nx, ny):
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
                elif di == 1:   # the E outflow face
                    A[r, r] += 1.5; A[r, idx(i - 1, j)] += -2; A[r, idx(i - 2, j)] += 0.5
            A[r, r] += d
    return A.tocsr()


# --- the closed operator D on (nx, ny) arrays, spacing h; E side face-Dirichlet if dE
def apply_d(z, h, dE):
    zp = np.pad(z, 1, mode="edge")                    # walls: ghost = value
    out = (zp[:-2, 1:-1] + zp[2:, 1:-1] + zp[1:-1, :-2] + zp[1:-1, 2:] - 4 * z) / h**2
    if dE:
        out[-1, :] -= 2 * z[-1, :] / h**2             # homogeneous face value
    return out


def diag_d(shape, h, dE):
    c = np.full(shape, 4.0)
    c[0, :] -= 1; c[-1, :] -= 1; c[:, 0] -= 1; c[:, -1] -= 1
    d = -c / h**2
    if dE:
        d[-1, :] -= 2 / h**2
    return d


def rbgs(z, b, h, dE, w, n):
    I, J = np.meshgrid(np.arange(z.shape[0]), np.arange(z.shape[1]), indexing="ij")
    dg = diag_d(z.shape, h, dE)
    for _ in range(n):
        for c in (0, 1):
            m = (I + J) % 2 == c
            z[m] += w * (b - apply_d(z, h, dE))[m] / dg[m]
    return z


def restrict(r):
    return 0.25 * (r[0::2, 0::2] + r[1::2, 0::2] + r[0::2, 1::2] + r[1::2, 1::2])


def prolong(e, dE):
    nxc, nyc = e.shape
    ep = np.pad(e, 1, mode="edge")                    # walls: even reflection
    if dE:
        ep[-1, :] = -ep[-2, :]                        # face-Dirichlet side: odd
    ep[:, 0] = ep[:, 1]; ep[:, -1] = ep[:, -2]
    f = np.zeros((2 * nxc, 2 * nyc))
    C = ep[1:-1, 1:-1]
    for a in (0, 1):
        for q in (0, 1):
            In = np.arange(nxc) + (2 if a else 0)
            Jn = np.arange(nyc) + (2 if q else 0)
            f[a::2, q::2] = (9 * C + 3 * ep[In][:, 1:-1] + 3 * ep[1:-1][:, Jn] + ep[In][:, Jn]) / 16
    return f


def vcycle(z, b, h, dE, w=1.15):
    if min(z.shape) <= 4:
        return rbgs(z, b, h, dE, 1.5, 60)
    z = rbgs(z, b, h, dE, w, 2)
    ec = vcycle(np.zeros((z.shape[0] // 2, z.shape[1] // 2)), restrict(b - apply_d(z, h, dE)), 2 * h, dE, w)
    return rbgs(z + prolong(ec, dE), b, h, dE, w, 2)


def closed_op(nx, ny):
    """D as a matrix (the line/exact variant): walls W, S, N; face-Dirichlet E."""
    idx = lambda i, j: i * ny + j
    T = sp.lil_matrix((nx * ny, nx * ny))
    for i in range(nx):
        for j in range(ny):
            r, d = idx(i, j), 0.0
            for di, dj in ((-1, 0), (1, 0), (0, -1), (0, 1)):
                ii, jj = i + di, j + dj
                if 0 <= ii < nx and 0 <= jj < ny:
                    T[r, idx(ii, jj)] = 1
                    d -= 1
                elif di == 1:
                    d -= 2
            T[r, r] = d
    return T.tocsc()


def lap1d_pinned(n):
    d = np.full(n, -2.0); d[0] = d[-1] = -1.0
    L = sp.diags([np.ones(n - 1), d, np.ones(n - 1)], [-1, 0, 1]).tolil()
    L[0, :] = 0
    L[0, 0] = 1.0
    return spla.splu(L.tocsc())


def main():
    rng = np.random.default_rng(0)
    for nx, ny in ((64, 32), (256, 64), (256, 128)):
        A = true_op(nx, ny)
        P = lambda v: v - v.mean()
        AP = spla.LinearOperator(A.shape, matvec=lambda v: P(A @ v))
        b = P(rng.uniform(-1, 1, nx * ny))
        luy = lap1d_pinned(ny)
        lu = spla.splu(closed_op(nx, ny))
        out = []
        for mode in ("wall", "line/exact", "line/v0", "line/vext"):
            def apply(r, mode=mode):
                r = np.asarray(r, dtype=float)
                if mode == "wall":
                    return P(vcycle(np.zeros((nx, ny)), r.reshape(nx, ny).copy(), 1.0, False).ravel())
                rE = r[(nx - 1) * ny:] - r[(nx - 1) * ny:].mean()
                rE[0] = 0.0
                g = luy.solve(rE)
                g -= g.mean()
                rr = r.copy()
                rr[(nx - 1) * ny:] -= 2 * g
                if mode == "line/exact":
                    return P(lu.solve(rr))
                z0 = np.zeros((nx, ny)) if mode == "line/v0" else np.tile(g, (nx, 1))
                return P(vcycle(z0, rr.reshape(nx, ny), 1.0, True).ravel())

            its = [0]
            spla.bicgstab(AP, b, M=spla.LinearOperator(A.shape, matvec=apply), rtol=1e-8, maxiter=3000,
                          callback=lambda xk: its.__setitem__(0, its[0] + 1))
            out.append(f"{mode} {its[0]}")
        print(f"{nx}x{ny}: " + ", ".join(out), flush=True)


if __name__ == "__main__":
    main()
