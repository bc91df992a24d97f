#!/bin/bash
# GPU suite on one variant library (LIB), then ab_lib over LIBS
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${OUT:-r03_ab2}
mkdir -p $out
if [ -n "$LIB" ]; then
  NSGPU_LIB=$LIB timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout=300 --timeout-method=thread ${TESTS:+-k "$TESTS"} > $out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest_gpu.log
  [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $out/pytest_gpu.log | head -30; exit 1; }
fi
bash tools/ab_lib.sh $LIBS || exit 1
[ -n "$PMC" ] && bash tools/ab_pmc.sh $LIBS
exit 0
