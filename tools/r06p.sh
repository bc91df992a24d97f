# lean band launch (weights per update, 68 VGPRs): identity check + kernel-trace A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
o=${1:-gpurun_out/r06p}
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_rccl.py tests/test_gpu_mask.py -k "band or loopback or mask" > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for m in 1 0; do
  NSGPU_BAND_LEAN=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace_$m -o run -- \
    python3 bench.py --warmup 5 --steps 20 --no-cpu --no-jacobi > $o/trace_$m.log 2>&1 || exit 1
  python3 tools/trace_summary.py $(find $o/trace_$m -name "*kernel_trace.csv" | head -1) 20 k_rhs@5 > $o/summary_$m.txt
  echo "== lean $m"; grep -E "band|total" $o/summary_$m.txt
done
