# mt v4 (branch-free relax): checks, L-shape A/B (bands 6 / 12, width 128 / 256) and trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
o=${1:-gpurun_out/r06m}
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_mask.py \
  -k "bit_identical or full_steps or wall_bands" > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for cfg in "6 128" "12 128" "6 256" "12 256" "0 128"; do
  set -- $cfg
  NSGPU_MASK_BAND=$1 NSGPU_MASK_BAND_W=$2 timeout -k 10 200 python -u tools/bench_bcs.py --lshape-only 4096 \
    > $o/lshape_band$1_w$2.log 2>&1 || exit 1
  echo "band $1 w $2: $(grep -h MLUPS $o/lshape_band$1_w$2.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace_lshape -o run -- \
  python3 tools/bench_bcs.py --lshape-only 4096 > $o/trace_lshape.log 2>&1 || exit 1
python3 tools/trace_summary.py $(find $o/trace_lshape -name "*kernel_trace.csv" | head -1) 3 k_rhs_lds@2 > $o/lshape_summary.txt
head -16 $o/lshape_summary.txt
