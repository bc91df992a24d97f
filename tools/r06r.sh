# capacitance solve into phi directly (masked inverse transform): checks + L-shape; the bench's timed-step phase.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
o=${1:-gpurun_out/r06r}
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_mask.py tests/test_gpu_fps.py \
  tests/test_gpu_rccl.py -k "mask or capacitance or cap or loopback" > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 200 python -u tools/bench_bcs.py --lshape-only 4096 > $o/lshape.log 2>&1 || exit 1
grep -h MLUPS $o/lshape.log
timeout -k 10 300 python -u bench.py --n 8192 --warmup 5 --steps 10 --no-cpu > $o/n8192.log 2>&1 || exit 1
python3 tools/bench_line.py n8192 $o/n8192.log
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --no-cpu --no-jacobi > $o/driver.log 2>&1 || exit 1
python3 tools/bench_line.py driver $o/driver.log
