#!/bin/bash
# 2x2-workgroup strip mapping (WG2X2): GPU suite on the variant library, then an interleaved A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${OUT:-r03_wg}
mkdir -p $out
L=navierstokessolver_amd
NSGPU_LIB=$L/libnsgpu_wg.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout=300 --timeout-method=thread ${TESTS:+-k "$TESTS"} > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $out/pytest_gpu.log | head -30; exit 1; }
bash tools/ab_lib.sh $L/libnsgpu.so $L/libnsgpu_wg.so $L/libnsgpu_wgntl.so
