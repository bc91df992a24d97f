#!/bin/bash
# coarse V-cycle check: phase timings, the multigrid / outflow / mask parity tests, bench A/B
# (NSGPU_CV_BLK 0 / 1) on the cavity and the channel, then the band-tuning windows
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${OUT:-r03_cv2}
mkdir -p $out
NSGPU_LIB=navierstokessolver_amd/libnsgpu_cvprof.so timeout -k 10 200 python3 bench.py --no-cpu --warmup 5 --steps 10 > $out/cvprof_1.log 2>&1 || exit $?
grep cvprof $out/cvprof_1.log | head -2 | cut -c1-600
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_mask.py \
  tests/test_gpu_multirank.py > $out/pytest.log 2>&1; rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for b in 0 1; do
    NSGPU_CV_BLK=$b timeout -k 10 200 python3 bench.py --no-cpu > $out/bench_${b}_$rep.log 2>&1 || exit $?
    python3 tools/bench_line.py "blk=$b" $out/bench_${b}_$rep.log
    NSGPU_CV_BLK=$b timeout -k 10 200 python3 bench.py --no-cpu --case channel > $out/chan_${b}_$rep.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$out/chan_${b}_$rep.log').read().strip().splitlines()[-1]); print('chan blk=$b', round(d['value']), round(d['ms_per_step'],3), d.get('poisson_bicgstab_its_per_step'))"
  done
done
if [ -n "$CONFIGS" ]; then OUT=${OUT:-r03_cv2}/band bash tools/r03_bandtune.sh || exit $?; fi
echo done
