#!/bin/bash
# one GPU session: the GPU suite (or a -k subset: TESTS=...), the default bench, then the
# developed-flow bench lines (tools/r03_devflow.sh) -- each step under its own time limit
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${OUT:-r03_check}
mkdir -p $out
sel=${TESTS:+-k "$TESTS"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout=300 --timeout-method=thread $sel > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $out/pytest_gpu.log | tail -3
[ $rc -gt 1 ] && exit $rc
[ $rc -eq 1 ] && { grep -E "^FAILED|Error" $out/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 300 python -u bench.py > $out/bench_default.log 2>&1 || exit $?
python3 tools/bench_line.py default $out/bench_default.log
[ -n "$NODEV" ] && exit 0
OUT=$(basename $out)/devflow bash tools/r03_devflow.sh
