#!/bin/bash
# wall-band sweep count at 8192^2 / 16384^2: bench lines per NSGPU_BAND_SWEEPS
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/bsw
for cfg in "8192 6" "8192 12" "16384 6" "16384 12"; do
  set -- $cfg
  w=$(( $1 >= 16384 ? 3 : 5 )); k=$(( $1 >= 16384 ? 4 : 10 ))
  NSGPU_BAND_SWEEPS=$2 timeout -k 10 300 python -u bench.py --n $1 --warmup $w --steps $k --no-cpu > gpurun_out/bsw/n$1_s$2.log 2>&1 || exit $?
  python3 tools/bench_line.py "n=$1 sweeps=$2" gpurun_out/bsw/n$1_s$2.log
done
