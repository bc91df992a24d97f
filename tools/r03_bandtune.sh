#!/bin/bash
# Helmholtz wall-band tuning in developed flow and at start-up: for each "NAME:ENV=VAL[,ENV=VAL]"
# in CONFIGS and each "warmup:steps" window in WINDOWS, the 4096^2 bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${OUT:-r03_bandtune}
mkdir -p $out
for cfg in ${CONFIGS:-base:}; do
  name=${cfg%%:*}; envs=${cfg#*:}
  for win in ${WINDOWS:-10:40 2000:40}; do
    w=${win%%:*}; k=${win#*:}
    ( [ -n "$envs" ] && export $(echo $envs | tr "," " ") ; timeout -k 10 200 python -u bench.py --no-cpu --warmup $w --steps $k --time-every 0 > $out/${name}_w${w}_s$k.log 2>&1 ) || exit $?
    python3 tools/bench_line.py "${name}_w${w}_s$k" $out/${name}_w${w}_s$k.log
  done
done
echo done
