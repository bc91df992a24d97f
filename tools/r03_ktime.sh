#!/bin/bash
# Per-kernel times of bench variants: for each "NAME:ENV=VAL[,ENV=VAL]" in VARIANTS, a rocprofv3
# kernel trace of a short bench (2 warm-up + 6 steps, --no-cpu) and the summary lines matching
# GREP (a regex).  Output under gpurun_out/$OUT/NAME.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${OUT:-r03_ktime}
mkdir -p $out
for v in ${VARIANTS:-base:}; do
  name=${v%%:*}; envs=${v#*:}
  ( [ -n "$envs" ] && export $(echo $envs | tr "," " ") ; timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/$name -o run -- python3 bench.py --no-cpu --warmup 2 --steps 6 --time-every 0 > $out/$name.log 2>&1 ) || exit $?
  python3 tools/trace_summary.py $(find $out/$name -name "*kernel_trace.csv" | head -1) 8 > $out/${name}_summary.txt
  echo "== $name: $(python3 tools/bench_line.py $name $out/$name.log)"
  grep -E "${GREP:-.}" $out/${name}_summary.txt | head -${TOP:-12}
done
echo done
