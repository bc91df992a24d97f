#!/bin/bash
# virtual-slab projections with the link-byte upper bound: 4096^2 (default agglomeration, and
# agglomerating from 256^2), 8192^2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r03_proj2; mkdir -p $out
timeout -k 10 400 python3 -u tools/slab_projection.py --n 4096 --ranks 1,2,4,8 > $out/projection_4096.log 2>&1 || exit $?
tail -1 $out/projection_4096.log
if [ -n "$AGG" ]; then
  NSGPU_AGG_CELLS=65536 timeout -k 10 400 python3 -u tools/slab_projection.py --n 4096 --ranks 1,2,4,8 > $out/projection_4096_agg256.log 2>&1 || exit $?
  tail -1 $out/projection_4096_agg256.log
fi
timeout -k 10 500 python3 -u tools/slab_projection.py --n 8192 --ranks 1,2,4,8 > $out/projection_8192.log 2>&1 || exit $?
tail -1 $out/projection_8192.log
