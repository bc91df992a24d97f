#!/bin/bash
# channel path check: outflow / apply parity tests, the channel bench (streaming apply vs the grid
# kernel, NSGPU_CELL=grid) with a kernel trace, the cavity bench, and a virtual P=2 slab trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${OUT:-r03_chan}
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "outflow or neumann or apply or stretched" > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for mode in stream grid; do
    e=""; [ $mode = grid ] && e="NSGPU_CELL=grid"
    env $e timeout -k 10 200 python3 bench.py --case channel --no-cpu --warmup 10 --steps 20 > $out/chan_${mode}_$rep.log 2>&1 || exit $?
    echo "$mode $(python3 tools/bench_line.py $mode $out/chan_${mode}_$rep.log)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/chan_trace -o run -- python3 bench.py --case channel --no-cpu --warmup 2 --steps 8 --time-every 0 > $out/chan_trace.log 2>&1 || exit $?
python3 tools/trace_summary.py $(find $out/chan_trace -name "*kernel_trace.csv" | head -1) 10 > $out/chan_per_step_summary.txt
head -16 $out/chan_per_step_summary.txt
timeout -k 10 200 python3 bench.py --no-cpu > $out/cavity.log 2>&1 || exit $?
echo "cavity $(python3 tools/bench_line.py cavity $out/cavity.log)"
OUT=${OUT:-r03_chan}/virt RANKS=2 TRACE_P=2 REPLAY=3:3,3:2,3:2 timeout -k 10 700 bash tools/r03_virtual.sh || exit $?
echo done
