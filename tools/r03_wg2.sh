#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r03_wg2
mkdir -p $out
L=navierstokessolver_amd
[ -n "$SKIPT" ] || NSGPU_LIB=$L/libnsgpu_wgup.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout=300 --timeout-method=thread > $out/pytest_gpu.log 2>&1
rc=$?; [ -n "$SKIPT" ] && rc=0; echo "pytest rc=$rc"; tail -3 $out/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $out/pytest_gpu.log | head -30; exit 1; }
bash tools/ab_lib.sh $L/libnsgpu.so $L/libnsgpu_wg.so $L/libnsgpu_wgup.so $L/libnsgpu_up.so || exit 1
bash tools/ab_pmc.sh $L/libnsgpu.so $L/libnsgpu_wg.so $L/libnsgpu_wgup.so || exit 1
STEPS=30 NSGPU_VERBOSE=1 timeout -k 10 120 python -u tools/verbose_steps.py > $out/verbose.log 2>&1
