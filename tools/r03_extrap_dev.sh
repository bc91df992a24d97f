#!/bin/bash
# phi extrapolation order in developed flow: bench lines after 300 / 2000 warm-up steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r03_extrap_dev; mkdir -p $out
for w in 300 2000; do for e in 2 3; do
  NSGPU_PHI_EXTRAP=$e timeout -k 10 200 python -u bench.py --no-cpu --warmup $w --steps 40 --time-every 0 > $out/bench_${e}_w$w.log 2>&1 || exit $?
  python3 tools/bench_line.py "e${e}_warmup_$w" $out/bench_${e}_w$w.log
done; done
