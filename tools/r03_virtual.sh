#!/bin/bash
# one rank's share of the multi-GPU step (virtual slab, tools/slab_projection.py) at N x N on P
# ranks: projection lines and a kernel trace (counted from the first K1 launch, so RCCL's
# communicator init is excluded).  N, RANKS (list for the projection), TRACE_P (ranks of the traced run)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
N=${N:-4096}
out=gpurun_out/${OUT:-r03_virtual}
mkdir -p $out
timeout -k 10 600 python3 -u tools/slab_projection.py --n $N --ranks ${RANKS:-1,2,4,8} ${PROJ_ARGS} > $out/projection_$N.log 2>&1 || exit $?
cat $out/projection_$N.log
if [ -n "$TRACE_P" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/p$TRACE_P -o run -- python3 tools/slab_projection.py --n $N --ranks $TRACE_P --replay ${REPLAY:-3:3,3:3} --warmup 2 --steps 6 > $out/p$TRACE_P.log 2>&1 || exit $?
  python3 tools/trace_summary.py $(find $out/p$TRACE_P -name "*kernel_trace.csv" | head -1) 8 k_rhs > $out/p${TRACE_P}_summary.txt
  head -45 $out/p${TRACE_P}_summary.txt
fi
echo done
