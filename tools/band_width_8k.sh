set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/b8k
for cfg in "128 6" "256 6" "256 9" "384 9"; do
  set -- $cfg
  NSGPU_BAND_W=$1 NSGPU_BAND_SWEEPS=$2 timeout -k 10 200 python -u bench.py --n 8192 --warmup 5 --steps 10 --no-cpu > gpurun_out/b8k/w$1_s$2.log 2>&1 || exit $?
  python3 tools/bench_line.py "w=$1 s=$2" gpurun_out/b8k/w$1_s$2.log
done
