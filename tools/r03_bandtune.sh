#!/bin/bash
# Helmholtz wall-band tuning in developed flow and at start-up: for each "NAME:ENV=VAL[,ENV=VAL]"
# in CONFIGS, the 4096^2 bench after 10 and 2000 warm-up steps (40 timed)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${OUT:-r03_bandtune}
mkdir -p $out
for cfg in ${CONFIGS:-base:}; do
  name=${cfg%%:*}; envs=${cfg#*:}
  for w in ${WARMUPS:-10 2000}; do
    ( [ -n "$envs" ] && export $(echo $envs | tr "," " ") ; timeout -k 10 200 python -u bench.py --no-cpu --warmup $w --steps 40 --time-every 0 > $out/${name}_w$w.log 2>&1 ) || exit $?
    python3 tools/bench_line.py "${name}_w$w" $out/${name}_w$w.log
  done
done
echo done
