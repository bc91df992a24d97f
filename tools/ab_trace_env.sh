#!/bin/bash
# kernel-trace A/B over environment settings: for each "NAME:ENV=VAL[,ENV=VAL]" a rocprofv3 kernel
# trace of the driver-form bench and the kernels matching $K (grep -E)
set -o pipefail
export TMPDIR=/tmp
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}; out=gpurun_out/ab_trace_env/$name; mkdir -p $out
  ( [ -n "$envs" ] && export $(echo $envs | tr "," " "); timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out -o run -- python3 bench.py --warmup 5 --steps 20 --no-cpu > $out/log 2>&1 ) || exit $?
  python3 tools/trace_summary.py $(find $out -name "*kernel_trace.csv" | head -1) 25 > $out/summary.txt
  echo "== $name: $(head -1 $out/summary.txt)"; grep -E "${K:-k_sweep3}" $out/summary.txt | tr -s ' ' | cut -c1-140
done
