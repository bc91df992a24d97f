# round-6 check: the whole GPU suite, then the deferred-K5 A/B (driver form, alternating NSGPU_K5_DEFER) and a
# kernel trace of the default.   gpurun -- bash tools/r06c_defer_ab.sh [outdir]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
o=${1:-gpurun_out/r06c}
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout=300 --timeout-method=thread \
  > $o/tests.log 2>&1
rc=$?
tail -3 $o/tests.log; grep -E "^FAILED" $o/tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for k in 1 2 3 4; do
  d=$((k % 2))
  NSGPU_K5_DEFER=$d timeout -k 10 200 python -u bench.py --warmup 5 --steps 20 --no-cpu --no-jacobi > $o/b$k.log 2>&1 || exit 1
  python3 tools/bench_line.py "defer$d" $o/b$k.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace -o run -- python3 bench.py --warmup 5 --steps 20 --no-cpu --no-jacobi > $o/trace.log 2>&1 || exit 1
python3 tools/trace_summary.py $(find $o/trace -name "*kernel_trace.csv" | head -1) 25 > $o/per_step_summary.txt
head -24 $o/per_step_summary.txt
