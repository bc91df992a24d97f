#!/bin/bash
# A/B session: a GPU-test subset (TESTS, a pytest -k expression), then bench lines for each
# "NAME:ENV=VAL[,ENV=VAL]" in VARIANTS (interleaved twice), then a kernel trace of the default
# bench (PROF=1).  Output under gpurun_out/$OUT.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${OUT:-r03_ab}
mkdir -p $out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout=300 --timeout-method=thread -k "$TESTS" > $out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $out/pytest_gpu.log | tail -3
  [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $out/pytest_gpu.log | head -30; exit 1; }
fi
for rep in 1 2; do
  for v in ${VARIANTS:-base:}; do
    name=${v%%:*}; envs=${v#*:}
    ( [ -n "$envs" ] && export $(echo $envs | tr "," " ") ; timeout -k 10 300 python -u bench.py --no-cpu ${BENCH_ARGS} > $out/bench_${name}_$rep.log 2>&1 ) || exit $?
    python3 tools/bench_line.py ${name}_$rep $out/bench_${name}_$rep.log
  done
done
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --no-cpu ${BENCH_ARGS} > $out/trace.log 2>&1 || exit $?
  python3 tools/trace_summary.py $(find $out/trace -name "*kernel_trace.csv" | head -1) 30 > $out/per_step_summary.txt
  head -40 $out/per_step_summary.txt
fi
echo done
