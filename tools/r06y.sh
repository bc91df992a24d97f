# The one-row real-input forward transform (k_fps_dct_div_r): fps / slab / loopback / parity checks, then same-box
# A/B traces (NSGPU_FPS_REAL 0 / 1) at 4096^2 and the sizes run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
o=${1:-gpurun_out/r06y}
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fps.py tests/test_gpu_rccl.py \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "row_transforms or outflow or direct or fused or fps or loopback or known_answer or deferred or bench_workload or slab" \
  > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for m in 0 1; do
  NSGPU_FPS_REAL=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace_$m -o run -- \
    python3 bench.py --warmup 5 --steps 20 --no-cpu --no-jacobi > $o/trace_$m.log 2>&1 || exit 1
  python3 tools/trace_summary.py $(find $o/trace_$m -name "*kernel_trace.csv" | head -1) 20 k_rhs@5 > $o/summary_$m.txt
  echo "== real $m"; grep -E "total|k_fps_dct|k_fps_idct" $o/summary_$m.txt
  rm -rf $o/trace_$m
done
for n in 8192 16384; do
  for m in 0 1; do
    NSGPU_FPS_REAL=$m timeout -k 10 300 python -u bench.py --n $n --warmup 3 --steps 10 --no-cpu --no-jacobi > $o/n${n}_$m.log 2>&1 || exit 1
    echo "n $n real $m"; python3 tools/bench_line.py sizes $o/n${n}_$m.log
  done
done
