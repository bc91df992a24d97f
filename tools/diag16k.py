import sys, numpy as np, scipy.fft as sf
sys.path.insert(0, '.'); sys.path.insert(0, 'oracle')
import navierstokessolver_amd as gpu
from oracle import OGrid
for nx, ny in [(64, 8192), (64, 16384)]:
    rng = np.random.default_rng(nx * 7 + ny)
    og = OGrid.rectangle(nx, ny, lx=nx / ny)
    gs = gpu.GpuSolver(gpu.rectangle(nx, ny, lx=nx / ny), 1e-3, 100.0, rtol=1.0)
    b = rng.uniform(-100, 100, nx * ny)
    gs.set(gpu.NS_ARR_PHI, np.zeros(nx * ny)); gs.set(gpu.NS_ARR_RPHI, b)
    its, res = gs.kernel(gpu.NS_K_POIS_SOLVE)[:2]
    g = gs.get(gpu.NS_ARR_PHI).ravel(); gs.close()
    bm = b - b.mean()
    r = (og.apply_poisson(g - g.mean()) - bm).reshape(nx, ny)
    x = og.fps_solve(b)
    print(nx, ny, "its", its, "lib res", res, "host res", np.linalg.norm(r) / np.linalg.norm(bm),
          "rel err vs oracle", np.max(np.abs((g - g.mean()) - (x - x.mean()))) / np.max(np.abs(x)))
    R = sf.dct(r, type=2, axis=1)
    e = np.sqrt((R ** 2).sum(axis=0))
    top = np.argsort(e)[::-1][:12]
    print("  worst modes", top.tolist(), (e[top] / np.linalg.norm(bm)).round(14).tolist())
    rowe = np.sqrt((r ** 2).sum(axis=1)) / np.linalg.norm(bm)
    print("  worst rows", np.argsort(rowe)[::-1][:8].tolist(), np.sort(rowe)[::-1][:4].tolist())
