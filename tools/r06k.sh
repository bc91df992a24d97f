# mt v2 (b prefetched, NEUMANN mask) check + L-shape A/B; traces of the driver-form bench and the L-shape.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
o=${1:-gpurun_out/r06k}
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_mask.py \
  tests/test_gpu_parity.py -k "bit_identical or full_steps or wall_bands or band" > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for cfg in "1 6" "1 0" "0 0"; do
  set -- $cfg
  NSGPU_MASK_MT=$1 NSGPU_MASK_BAND=$2 timeout -k 10 200 python -u tools/bench_bcs.py --lshape-only 4096 \
    > $o/lshape_mt$1_band$2.log 2>&1 || exit 1
  echo "mt $1 band $2: $(grep -h MLUPS $o/lshape_mt$1_band$2.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace_lshape -o run -- \
  python3 tools/bench_bcs.py --lshape-only 4096 > $o/trace_lshape.log 2>&1 || exit 1
python3 tools/trace_summary.py $(find $o/trace_lshape -name "*kernel_trace.csv" | head -1) 3 k_rhs_lds@2 > $o/lshape_summary.txt
head -24 $o/lshape_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace_base -o run -- \
  python3 bench.py --warmup 5 --steps 20 --no-cpu --no-jacobi > $o/trace_base.log 2>&1 || exit 1
python3 tools/trace_summary.py $(find $o/trace_base -name "*kernel_trace.csv" | head -1) 20 k_rhs@5 > $o/base_summary.txt
head -14 $o/base_summary.txt
timeout -k 10 200 python -u bench.py --warmup 5 --steps 20 --no-cpu --no-jacobi > $o/bench.log 2>&1 || exit 1
python3 tools/bench_line.py base $o/bench.log
