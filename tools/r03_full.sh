#!/bin/bash
# round-3 checkpoint: the whole GPU suite, the default bench (+ its rocprofv3 kernel trace), the
# projections (4096^2 and 8192^2 strong, 2048 x 8192 weak per rank); each step time-limited
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${OUT:-r03_full}
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout=300 --timeout-method=thread > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $out/pytest_gpu.log | tail -2; grep -E "^FAILED" $out/pytest_gpu.log | head
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u bench.py > $out/bench_default.log 2>&1 || exit $?
python3 tools/bench_line.py default $out/bench_default.log
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 > $out/bench_driver.log 2>&1 || exit $?
python3 tools/bench_line.py driver_form $out/bench_driver.log
[ -n "$NOPROF" ] || { timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/bench_trace -o run -- python3 bench.py --no-cpu > $out/bench_trace.log 2>&1 || exit $?; python3 tools/trace_summary.py $(find $out/bench_trace -name "*kernel_trace.csv" | head -1) 30 k_rhs > $out/bench_per_step_summary.txt; head -12 $out/bench_per_step_summary.txt; }
[ -n "$NOPROJ" ] && exit 0
timeout -k 10 600 python3 -u tools/slab_projection.py --n 4096 > $out/projection_4096.log 2>&1 || exit $?
tail -1 $out/projection_4096.log
timeout -k 10 600 python3 -u tools/slab_projection.py --n 8192 > $out/projection_8192.log 2>&1 || exit $?
tail -1 $out/projection_8192.log
timeout -k 10 900 python3 -u tools/slab_projection.py --weak-rows 2048 --ny 8192 --warmup 3 --steps 5 > $out/projection_weak.log 2>&1 || exit $?
tail -1 $out/projection_weak.log
echo done
