# branch-free chunk loads in the recurrences: direct-solve checks + driver-form bench + trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
o=${1:-gpurun_out/r06s}
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fps.py tests/test_gpu_parity.py \
  -k "direct or outflow or deferred or known_answer" > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --no-cpu --no-jacobi > $o/driver.log 2>&1 || exit 1
python3 tools/bench_line.py driver $o/driver.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace -o run -- \
  python3 bench.py --warmup 5 --steps 20 --no-cpu --no-jacobi > $o/trace.log 2>&1 || exit 1
python3 tools/trace_summary.py $(find $o/trace -name "*kernel_trace.csv" | head -1) 20 k_rhs@5 > $o/summary.txt
head -20 $o/summary.txt
