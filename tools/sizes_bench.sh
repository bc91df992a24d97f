#!/bin/bash
# bench lines at the other config sizes on one GPU (DESIGN 6 "Larger grids"): 2048^2 (configs[1]),
# 8192^2 and 16384^2 cavities, fp64, no CPU leg; one log each under gpurun_out/sizes/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/sizes
timeout -k 10 200 python -u bench.py --n 2048 --warmup 10 --steps 20 --no-cpu > gpurun_out/sizes/n2048.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --n 8192 --warmup 5 --steps 10 --no-cpu > gpurun_out/sizes/n8192.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --n 16384 --warmup 3 --steps 4 --no-cpu > gpurun_out/sizes/n16384.log 2>&1 || exit $?
echo done
