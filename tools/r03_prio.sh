#!/bin/bash
# env A/B on the virtual-slab projection (4096^2 by default, P = 1,2,4,8): for each
# "NAME:ENV=VAL[,ENV=VAL]" in CONFIGS, tools/slab_projection.py under that environment; then
# (LIBS set) an A/B of variant libraries on the bench workload
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${OUT:-r03_prio}
mkdir -p $out
for cfg in ${CONFIGS:-base:}; do
  name=${cfg%%:*}; envs=${cfg#*:}
  ( [ -n "$envs" ] && export $(echo $envs | tr "," " ") ; timeout -k 10 400 python3 -u tools/slab_projection.py --n ${N:-4096} --ranks ${RANKS:-1,2,4,8} \
    >> $out/projection_$name.log 2>&1 ) || exit $?
  echo "== $name"; tail -5 $out/projection_$name.log | cut -c1-200
done
if [ -n "$LIBS" ]; then
  timeout -k 10 900 bash tools/ab_lib.sh $LIBS || exit $?
fi
echo done
