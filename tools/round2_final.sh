#!/bin/bash
# round-2 closing evidence into gpurun_out/r02f/: the GPU suite, the default bench, its kernel trace,
# the FETCH / WRITE PMC passes (tools/round2_profile.sh), then the channel bench (bench.py --case
# channel) and its kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${OUT:-r02f}
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout=300 --timeout-method=thread > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $out/pytest_gpu.log | tail -3
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u bench.py > $out/bench_default.log 2>&1 || exit $?
tail -c 400 $out/bench_default.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/bench_trace -o run -- python3 bench.py --no-cpu > $out/bench_trace.log 2>&1 || exit $?
python3 tools/trace_summary.py $(find $out/bench_trace -name "*kernel_trace.csv" | head -1) 30 > $out/bench_per_step_summary.txt
bash tools/profile_round.sh $out/prof || exit $?
timeout -k 10 200 python -u bench.py --case channel > $out/bench_channel.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/channel_trace -o run -- python3 bench.py --case channel > $out/channel_trace.log 2>&1 || exit $?
python3 tools/trace_summary.py $(find $out/channel_trace -name "*kernel_trace.csv" | head -1) 30 > $out/channel_per_step_summary.txt
timeout -k 10 600 python -u tools/slab_projection.py > $out/projection.log 2>&1 || exit $?
cat $out/projection.log | tail -5
echo done
