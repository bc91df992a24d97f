#!/bin/bash
# Multi-rank rehearsal of the production shape on ONE GPU: N host-transport ranks (gloo) run the
# 4096^2 cavity with NSGPU_VERBOSE hierarchy output; the per-step monitor values are compared
# with a single-rank run.  Usage (GPU box): bash tools/mr_rehearse.sh [nproc] [n] [steps]
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
np=${1:-4}; n=${2:-4096}; steps=${3:-2}
mkdir -p gpurun_out
NSGPU_VERBOSE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$np \
  --master-addr=127.0.0.1 --master-port=29650 tests/mr_worker.py --xport host --size $n --nsteps $steps \
  --solver 2 --tol 1e-8 --stats-only --output gpurun_out/mr_rehearse.npz > gpurun_out/mr_rehearse.log 2>&1
grep -E "nsgpu mg|coarse" gpurun_out/mr_rehearse.log | sort -u | head -20
timeout -k 10 120 python - <<PY
import sys, numpy as np
sys.path.insert(0, ".")
import navierstokessolver_amd as nsa
r = np.load("gpurun_out/mr_rehearse.npz", allow_pickle=False)
print("status", r["status"])
gs = nsa.GpuSolver(nsa.rectangle($n, $n), 1.0 / (8 * $n), 100.0, device=0, rtol=1e-8)
mm = np.array([list(gs.step().values())[:7] for _ in range($steps)])
print("multi-rank:", r["mm"])
print("single    :", mm)
print("max |d monitor|", np.max(np.abs(r["mm"][:, :4] - mm[:, :4])))
PY
