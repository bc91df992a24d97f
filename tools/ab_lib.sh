#!/bin/bash
# A/B two or more builds of libnsgpu.so on the bench workload (run on the GPU box from the repo
# root):  bash tools/ab_lib.sh abl/libnsgpu_head.so navierstokessolver_amd/libnsgpu.so
# Each library runs twice, interleaved; prints value, ms/step and the timed kernels' averages.
set -e
mkdir -p gpurun_out
for rep in 1 2; do
  k=0
  for lib in "$@"; do
    k=$((k + 1))
    NSGPU_LIB=$lib timeout -k 10 200 python bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-10} --no-cpu \
      > gpurun_out/ablib_${k}_$rep.log 2>&1
    python3 -c "
import json; d=json.loads(open('gpurun_out/ablib_${k}_$rep.log').read().strip().splitlines()[-1])
ks=' '.join(f'{n}={v[\"avg_kernel_us\"]:.1f}us/{v[\"frac\"]:.3f}' for n, v in d['kernels'].items())
print('$lib', round(d['value']), round(d['ms_per_step'], 3), d['poisson_vcycles_per_step'], ks)"
  done
done
