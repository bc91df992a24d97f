# Row transforms' twiddles up front (FPS_RTW) and the reductions' shuffle tail: checks, then same-box A/B against the
# FPS_RTW=0 build (libnsgpu_nortw.so) at 4096^2 (kernel trace) and 8192^2 / 16384^2 (bench lines).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
o=${1:-gpurun_out/r06aa}
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fps.py tests/test_gpu_rccl.py \
  tests/test_gpu_parity.py -k "row_transforms or direct_solve_matches or fused or loopback or known_answer or deferred or 16384" \
  > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for lib in navierstokessolver_amd/libnsgpu_nortw.so navierstokessolver_amd/libnsgpu.so; do
  k=$(basename $lib .so)
  NSGPU_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace_$k -o run -- \
    python3 bench.py --warmup 5 --steps 20 --no-cpu --no-jacobi > $o/trace_$k.log 2>&1 || exit 1
  python3 tools/trace_summary.py $(find $o/trace_$k -name "*kernel_trace.csv" | head -1) 20 k_rhs@5 > $o/summary_$k.txt
  echo "== $k"; grep -E "total|k_fps_dct|k_fps_idct|reduce" $o/summary_$k.txt
  rm -rf $o/trace_$k
done
for n in 8192 16384; do
  for lib in navierstokessolver_amd/libnsgpu_nortw.so navierstokessolver_amd/libnsgpu.so; do
    k=$(basename $lib .so)
    NSGPU_LIB=$lib timeout -k 10 300 python -u bench.py --n $n --warmup 3 --steps 10 --no-cpu --no-jacobi > $o/n${n}_$k.log 2>&1 || exit 1
    echo "n $n $k"; python3 tools/bench_line.py sizes $o/n${n}_$k.log
  done
done
