#!/bin/bash
# A/B one environment knob on the bench workload (run on the GPU box from the repo root):
#   bash tools/ab_env.sh NSGPU_PHI_EXTRAP 1 2      -> value, V-cycles/step, Helmholtz sweeps/step per setting
# Each setting runs twice, interleaved, so drift between runs shows up.
set -e
var=$1; shift
mkdir -p gpurun_out
for rep in 1 2; do
  for val in "$@"; do
    env "$var=$val" timeout -k 10 200 python bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-10} --no-cpu \
      > gpurun_out/ab_${val}_$rep.log 2>&1
    python3 tools/bench_line.py "$var=$val" gpurun_out/ab_${val}_$rep.log
  done
done
