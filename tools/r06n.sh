# masked: no phi extrapolation under the capacitance solve, cell-kernel rows A/B; mask suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
o=${1:-gpurun_out/r06n}
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_mask.py > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -2 $o/tests.log
grep -h "full_steps" $o/tests.log | head -20
for r in 0 1 2 4 8; do
  NSGPU_CELL_ROWS=$r timeout -k 10 200 python -u tools/bench_bcs.py --lshape-only 4096 > $o/lshape_rows$r.log 2>&1 || exit 1
  echo "rows $r: $(grep -h MLUPS $o/lshape_rows$r.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace_lshape -o run -- \
  python3 tools/bench_bcs.py --lshape-only 4096 > $o/trace_lshape.log 2>&1 || exit 1
python3 tools/trace_summary.py $(find $o/trace_lshape -name "*kernel_trace.csv" | head -1) 3 k_rhs_lds@2 > $o/lshape_summary.txt
head -20 $o/lshape_summary.txt
