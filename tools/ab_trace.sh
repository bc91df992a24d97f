#!/bin/bash
# kernel-trace A/B: for each library, a rocprofv3 kernel trace of the driver-form bench and the
# average duration of the kernels matching $K (a grep -E pattern)
set -o pipefail
export TMPDIR=/tmp
k=0
for lib in "$@"; do
  k=$((k + 1)); out=gpurun_out/ab_trace/$k; mkdir -p $out
  NSGPU_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out -o run -- python3 bench.py --warmup 5 --steps 20 --no-cpu > $out/log 2>&1 || exit $?
  python3 tools/trace_summary.py $(find $out -name "*kernel_trace.csv" | head -1) 25 > $out/summary.txt
  echo "$lib: $(grep -E "${K:-k_axpby}" $out/summary.txt | tr -s ' ' | cut -c1-150)"
done
