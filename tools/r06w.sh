# K1's wall-ring workgroups first: checks (K1 / deferred / slabs / masked / idct mask) + A/B traces.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
o=${1:-gpurun_out/r06w}
mkdir -p $o
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_rccl.py \
  tests/test_gpu_multirank.py tests/test_gpu_fps.py -k "k1 or rhs or deferred or known_answer or slab or loopback or capacitance" \
  > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for m in 0 1; do
  NSGPU_K1_RING_LAST=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace_$m -o run -- \
    python3 bench.py --warmup 5 --steps 20 --no-cpu --no-jacobi > $o/trace_$m.log 2>&1 || exit 1
  python3 tools/trace_summary.py $(find $o/trace_$m -name "*kernel_trace.csv" | head -1) 20 k_rhs@5 > $o/summary_$m.txt
  echo "== ring_last $m"; grep -E "total|k_rhs" $o/summary_$m.txt
done
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --no-cpu --no-jacobi > $o/driver.log 2>&1 || exit 1
python3 tools/bench_line.py driver $o/driver.log
