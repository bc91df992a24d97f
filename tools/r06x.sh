# K1's wall ring: its share of the launch (timing probe without it: wrong results, timing only), same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
o=${1:-gpurun_out/r06x}
mkdir -p $o
for m in 0 1 0; do
  NSGPU_K1_PROBE_NORING=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace_$m -o run -- \
    python3 bench.py --warmup 5 --steps 20 --no-cpu --no-jacobi > $o/trace_$m.log 2>&1 || exit 1
  python3 tools/trace_summary.py $(find $o/trace_$m -name "*kernel_trace.csv" | head -1) 20 k_rhs@5 > $o/summary_$m.txt
  echo "== noring $m"; grep -E "total|k_rhs" $o/summary_$m.txt
  rm -rf $o/trace_$m
done
