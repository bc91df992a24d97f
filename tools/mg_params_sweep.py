"""4096^2 bench workload at several multigrid (pre, post, smoother omega) settings:
ms/step and V-cycles/step (one process; NSGPU_MG_OMEGA is read at solver creation)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import navierstokessolver_amd as nsa

n = int(os.environ.get("N", "4096"))
for pre, post in ((2, 2), (4, 2), (2, 4), (4, 4)):
    for w in (1.0, 1.05, 1.1, 1.15):
        os.environ["NSGPU_MG_OMEGA"] = str(w)
        s = nsa.GpuSolver(nsa.cavity(n), 1.0 / (8 * n), 1000.0, mg_pre=pre, mg_post=post)
        for _ in range(int(os.environ.get("W", "10"))):
            s.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        K = int(os.environ.get("K", "20"))
        st = [s.step() for _ in range(K)]
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / K
        print(f"pre={pre} post={post} omega={w:4.2f}: {t*1e3:6.3f} ms/step "
              f"{sum(x['it_phi'] for x in st)/K:4.2f} V-cycles/step", flush=True)
        s.close()
