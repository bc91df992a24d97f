#!/bin/bash
# phi extrapolation order A/B: per-step V-cycle counts (30 steps) and bench lines (driver form W=5 and default W=10)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r03_extrap; mkdir -p $out
for e in ${ORDERS:-2 3}; do
  NSGPU_PHI_EXTRAP=$e STEPS=${STEPS:-30} timeout -k 10 120 python -u tools/verbose_steps.py > $out/steps_$e.log 2>&1 || exit 1
  echo "extrap $e: $(grep '^step' $out/steps_$e.log | awk '{printf "%s ", $4}')"
done
for rep in 1 2; do for e in ${ORDERS:-2 3}; do for w in ${WS:-5 10}; do
  NSGPU_PHI_EXTRAP=$e timeout -k 10 200 python -u bench.py --no-cpu --warmup $w > $out/bench_${e}_${w}_$rep.log 2>&1 || exit 1
  python3 tools/bench_line.py e${e}_w${w}_$rep $out/bench_${e}_${w}_$rep.log
done; done; done
