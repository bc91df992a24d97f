#!/bin/bash
# closing session: full GPU suite, then tools/r03_final.sh (bench lines, trace, PMC)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${OUT:-r03_final}; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout=300 --timeout-method=thread > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $out/pytest_gpu.log | head -30; exit 1; }
bash tools/r03_final.sh
