# masked streaming K3 / K5: checks, L-shape A/B and trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
o=${1:-gpurun_out/r06o}
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_mask.py \
  tests/test_gpu_parity.py -k "mask or k3 or k5 or correct or div or deferred" > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for c in 1 0; do
  NSGPU_MASK_CELL=$c timeout -k 10 200 python -u tools/bench_bcs.py --lshape-only 4096 > $o/lshape_cell$c.log 2>&1 || exit 1
  echo "cell $c: $(grep -h MLUPS $o/lshape_cell$c.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace_lshape -o run -- \
  python3 tools/bench_bcs.py --lshape-only 4096 > $o/trace_lshape.log 2>&1 || exit 1
python3 tools/trace_summary.py $(find $o/trace_lshape -name "*kernel_trace.csv" | head -1) 3 k_rhs_lds@2 > $o/lshape_summary.txt
head -24 $o/lshape_summary.txt
