#!/bin/bash
# A/B library builds (make variant) on the bench workload with the kernel trace (run on the GPU box from the repo
# root):  bash tools/ab_lib_trace.sh <outdir> <kernel regex> lib1.so lib2.so ...
# per library: the bench line (value, ms/step, the last step's monitor -- equal when the variant is exact) and the
# matching kernels' per-step summary lines
set -e
out=$1; pat=$2; shift 2
export TMPDIR=/tmp
mkdir -p $out
k=0
for lib in "$@"; do
  k=$((k + 1))
  NSGPU_LIB=$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-jacobi > $out/bench_$k.json 2> $out/bench_$k.err
  python3 -c "
import json; d=json.loads(open('$out/bench_$k.json').read().strip().splitlines()[-1]); print('$lib', round(d['value']), round(d['ms_per_step'], 4), d['monitor_last_step'])"
done
k=0
for lib in "$@"; do
  k=$((k + 1))
  NSGPU_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_$k -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu --no-jacobi > $out/trace_$k.log 2>&1
  python3 tools/trace_summary.py $(find $out/trace_$k -name "*kernel_trace.csv" | head -1) 13 > $out/summary_$k.txt
  echo "== $lib"; grep -E "total|$pat" $out/summary_$k.txt || true
done
