#!/bin/bash
# A/B an environment knob on the bench workload with the kernel trace (run on the GPU box from the repo root):
#   bash tools/ab_env_trace.sh <outdir> VAR v1 v2 ...
# per value: the bench line (value, ms/step) and the per-step kernel summary (tools/trace_summary.py)
set -e
out=$1; var=$2; shift 2
export TMPDIR=/tmp
mkdir -p $out
for v in "$@"; do
  env $var=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu > $out/bench_$v.json 2> $out/bench_$v.err
  python3 -c "
import json; d=json.loads(open('$out/bench_$v.json').read().strip().splitlines()[-1]); print('$var=$v', round(d['value']), round(d['ms_per_step'], 4))"
done
for v in "$@"; do
  export $var=$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_$v -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu --no-jacobi > $out/trace_$v.log 2>&1
  python3 tools/trace_summary.py $(find $out/trace_$v -name "*kernel_trace.csv" | head -1) 13 > $out/summary_$v.txt
  echo "== $var=$v"; head -14 $out/summary_$v.txt
done
