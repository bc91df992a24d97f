"""Diagnostics: run cavity steps at several sizes, report sweeps / residuals, and
find the first stage that produces non-finite values."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import navierstokessolver_amd as nsa

def finite(gs, names):
    out = {}
    for nm in names:
        a = gs.get(getattr(nsa, "NS_ARR_" + nm))
        out[nm] = (bool(np.isfinite(a).all()), float(np.nanmax(np.abs(a))))
    return out

for n in [int(x) for x in sys.argv[1:]] or [512, 1024, 2048, 4096]:
    for timing in (False, True):
        gs = nsa.GpuSolver(nsa.cavity(n), 1.0 / (8 * n), 1000.0, timing=timing)
        t0 = time.time()
        try:
            for k in range(2):
                st = gs.step()
                print(f"n={n} timing={timing} step {k+1}: it_u={st['it_u']} it_phi={st['it_phi']} res_phi={st['res_phi']:.2e} "
                      f"umax={st['umax']:.6f} checks={st['n_checks']} t={time.time()-t0:.2f}s", flush=True)
        except nsa.NsError as e:
            print(f"n={n} timing={timing} FAILED: {e}", flush=True)
            gs2 = nsa.GpuSolver(nsa.cavity(n), 1.0 / (8 * n), 1000.0)
            gs2.kernel(nsa.NS_K_RHS); print("  after K1:", finite(gs2, ["RU", "RV", "CU", "CV"]), flush=True)
            o = gs2.kernel(nsa.NS_K_HELM_SOLVE); print("  helm solve its/res:", o[:2], finite(gs2, ["U", "V"]), flush=True)
            o = gs2.kernel(nsa.NS_K_DIV); print("  div sums:", o[:2], finite(gs2, ["RPHI"]), flush=True)
            for it in (1, 2, 4, 8, 16, 64, 256):
                o = gs2.kernel(nsa.NS_K_POISSON, it); print(f"  +{it} poisson sweeps: r2={o[0]:.3e}", finite(gs2, ["PHI"]), flush=True)
        gs.close()
