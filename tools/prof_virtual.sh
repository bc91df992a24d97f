#!/bin/bash
# kernel trace of one rank's share of the 8192^2 step on 8 GPUs (virtual slab) and of the
# single-GPU step, for the strong-scaling breakdown
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=${1:-gpurun_out/pv}
mkdir -p $out
for P in ${RANKS:-8 1}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p$P -o run -- python3 tools/slab_projection.py --ranks $P --replay 10:3,12:4 --warmup 3 --steps 6 > $out/p$P.log 2>&1
  rc=$?; echo "P=$P rc=$rc"; grep '"P"' $out/p$P.log
  [ $rc -ne 0 ] && exit $rc
  python3 tools/trace_summary.py $(find $out/p$P -name "*kernel_trace.csv" | head -1) 9 > $out/p${P}_summary.txt 2>&1
  head -40 $out/p${P}_summary.txt; python3 tools/gaps.py $(find $out/p$P -name "*kernel_trace.csv" | head -1) > $out/p${P}_gaps.txt 2>&1; head -30 $out/p${P}_gaps.txt
done
exit 0
