# A/B of strip / grid shapes (env knobs) on the driver-form bench, interleaved.  gpurun -- bash tools/r06g_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
o=${1:-gpurun_out/r06g}
mkdir -p $o
run() {   # run <label> <env...>
  local lab=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --warmup 5 --steps 20 --no-cpu --no-jacobi > $o/$lab.log 2>&1 || return 1
  python3 tools/bench_line.py "$lab" $o/$lab.log
}
for rep in 1 2; do
  run base$rep NSGPU_NOP=1 || exit 1
  run k1l16_$rep NSGPU_K1_L=16 || exit 1
  run k1l32_$rep NSGPU_K1_L=32 || exit 1
  run fpsg4k_$rep NSGPU_FPS_GRID=4096 || exit 1
  run fpsg256_$rep NSGPU_FPS_GRID=256 || exit 1
done
