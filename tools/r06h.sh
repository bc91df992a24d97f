# band6 + masked multi-sweep checks, then A/B of the band form / masked Helmholtz / strip shapes.  gpurun -- bash tools/r06h.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
o=${1:-gpurun_out/r06h}
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_mask.py -k "band or deferred or known_answer or helm or bit_identical or full_steps" \
  > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -2 $o/tests.log
NSGPU_MASK_MT=1 timeout -k 10 200 python -u tools/bench_bcs.py --lshape-only 4096 > $o/lshape_mt1.log 2>&1 || exit 1
NSGPU_MASK_MT=0 timeout -k 10 200 python -u tools/bench_bcs.py --lshape-only 4096 > $o/lshape_mt0.log 2>&1 || exit 1
grep -h "MLUPS" $o/lshape_mt1.log $o/lshape_mt0.log
run() {   # run <label> <env...>
  local lab=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --warmup 5 --steps 20 --no-cpu --no-jacobi > $o/$lab.log 2>&1 || return 1
  python3 tools/bench_line.py "$lab" $o/$lab.log
}
for rep in 1 2; do
  run base$rep NSGPU_NOP=1 || exit 1
  run band3_$rep NSGPU_BAND6=0 || exit 1
  run k1l16_$rep NSGPU_K1_L=16 || exit 1
  run fpsg4k_$rep NSGPU_FPS_GRID=4096 || exit 1
done
