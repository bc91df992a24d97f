#  steady-state kernel traces of the 4096^2 virtual slabs, P = 2 / 4 / 8 (warm-up excluded),
# with the idle gaps between kernels; then the strong-scaling projections.  gpurun -- bash tools/r06i.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
o=${1:-gpurun_out/r06i}
mkdir -p $o
for P in 8 4 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/vslab_p${P} -o run -- \
    python3 tools/vslab_trace.py 4096 $P > $o/vslab_p${P}.log 2>&1 || exit 1
  f=$(find $o/vslab_p${P} -name "*kernel_trace.csv" | head -1)
  python3 tools/trace_summary.py $f 20 k_rhs@5 > $o/vslab_p${P}_4096_summary.txt
  python3 tools/gaps.py $f 300 > $o/vslab_p${P}_4096_gaps.txt
  head -30 $o/vslab_p${P}_4096_summary.txt; head -8 $o/vslab_p${P}_4096_gaps.txt; tail -1 $o/vslab_p${P}.log
done
