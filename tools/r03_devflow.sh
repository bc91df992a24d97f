#!/bin/bash
# developed-flow vs start-up numbers of the default bench: the same 4096^2
# cavity after 5 / 10 / 2000 / 4000 warm-up steps, with and without the Helmholtz wall bands
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${OUT:-r03_devflow}
mkdir -p $out
for w in 5 10 2000 4000; do
  timeout -k 10 200 python -u bench.py --no-cpu --warmup $w --steps 40 --time-every 0 > $out/bench_w$w.log 2>&1 || exit $?
  python3 tools/bench_line.py "warmup_$w" $out/bench_w$w.log
done
for w in 10 2000; do
  NSGPU_HELM_BAND=0 timeout -k 10 200 python -u bench.py --no-cpu --warmup $w --steps 40 --time-every 0 > $out/bench_noband_w$w.log 2>&1 || exit $?
  python3 tools/bench_line.py "noband_warmup_$w" $out/bench_noband_w$w.log
done
echo done
