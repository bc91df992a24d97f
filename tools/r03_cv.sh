#!/bin/bash
# coarse V-cycle A/B: phase timings (CV_PROF build) of the cell-loop and 2x2-block smoothers,
# the multigrid parity tests, interleaved bench runs, then the PMC passes of tools/profile_round.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${OUT:-r03_cv}
mkdir -p $out
for b in 0 1; do
  NSGPU_CV_BLK=$b NSGPU_LIB=navierstokessolver_amd/libnsgpu_cvprof.so timeout -k 10 200 python3 bench.py --no-cpu --warmup 5 --steps 10 > $out/cvprof_$b.log 2>&1 || exit $?
  echo "blk=$b"; grep cvprof $out/cvprof_$b.log | head -3 | cut -c1-600
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_mask.py \
  > $out/pytest.log 2>&1; rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for b in 0 1; do
    NSGPU_CV_BLK=$b timeout -k 10 200 python3 bench.py --no-cpu > $out/bench_${b}_$rep.log 2>&1 || exit $?
    python3 tools/bench_line.py "blk=$b" $out/bench_${b}_$rep.log
  done
done
[ -n "$PROF" ] && bash tools/profile_round.sh $out/prof && cat $out/prof/valu_per_cell.json
echo done
