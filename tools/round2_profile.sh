#!/bin/bash
# r02 evidence: the full GPU suite, the default bench, its rocprofv3 kernel-trace --stats, and the
# FETCH / WRITE PMC passes (tools/profile_round.sh) into gpurun_out/r02/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r02
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout=300 --timeout-method=thread > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $out/pytest_gpu.log | tail -3
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u bench.py > $out/bench_default.log 2>&1 || exit $?
tail -c 600 $out/bench_default.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/bench_trace -o run -- python3 bench.py --no-cpu > $out/bench_trace.log 2>&1 || exit $?
python3 tools/trace_summary.py $(find $out/bench_trace -name "*kernel_trace.csv" | head -1) 30 > $out/bench_per_step_summary.txt
head -12 $out/bench_per_step_summary.txt
bash tools/profile_round.sh $out/prof || exit $?
cat $out/prof/pmc_traffic.json
