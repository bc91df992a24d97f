#!/bin/bash
# GPU suite, then bench lines: driver form (W=5), default (W=10), developed flow (W=300, 2000)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${OUT:-r03_check2}; mkdir -p $out
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout=300 --timeout-method=thread ${TESTS:+-k "$TESTS"} > $out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest_gpu.log
  [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $out/pytest_gpu.log | head -30; exit 1; }
fi
for w in 5 10 300 2000; do
  timeout -k 10 200 python -u bench.py --no-cpu --warmup $w > $out/bench_w$w.log 2>&1 || exit $?
  python3 tools/bench_line.py "warmup_$w" $out/bench_w$w.log
done
