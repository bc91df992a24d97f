#!/bin/bash
# The GPU evidence behind DESIGN.md, one mode per kind of record (run on the GPU box from the repo
# root, e.g. `gpurun -- bash tools/evidence.sh bench gpurun_out/r04_x`); every GPU step has its own
# time limit and the steps are chained so that the first failure ends the call.
#   suite       the whole `pytest -m gpu` suite                               -> pytest_gpu.log
#   bench       the default bench line and the driver's form (5 + 20 steps), both with the CPU leg,
#               and a rocprofv3 kernel trace of the driver's form              -> bench_*.log, per_step_summary.txt
#   pmc         rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE, VALU) of the bench -> profile_round.sh
#   sizes       bench lines at 2048^2 (configs[1]), 8192^2, 16384^2 (no CPU leg)
#   projection  virtual-slab projections: 4096^2 and 8192^2 strong, 2048 x 8192 per rank weak
#   devflow     the default bench after 5 / 10 / 2000 warm-up steps (start-up vs developed flow)
#   jacobi      the Jacobi sweep benchmark at 4096^2 / 8192^2 / 16384^2, fp64 and fp32 (sweep_c5.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mode=$1
out=${2:-gpurun_out/ev_$mode}
mkdir -p $out
line() { python3 tools/bench_line.py "$1" "$2"; }
case $mode in
suite)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout=300 --timeout-method=thread \
    > $out/pytest_gpu.log 2>&1
  rc=$?; grep -E "passed|failed" $out/pytest_gpu.log | tail -2; grep -E "^FAILED" $out/pytest_gpu.log | head
  exit $rc ;;
bench)
  timeout -k 10 400 python -u bench.py > $out/bench_default.log 2>&1 || exit $?
  line default $out/bench_default.log
  timeout -k 10 400 python -u bench.py --warmup 5 --steps 20 > $out/bench_driver_form.log 2>&1 || exit $?
  line driver_form $out/bench_driver_form.log
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
    python3 bench.py --warmup 5 --steps 20 --no-cpu > $out/trace.log 2>&1 || exit $?
  python3 tools/trace_summary.py $(find $out/trace -name "*kernel_trace.csv" | head -1) 25 > $out/per_step_summary.txt
  head -16 $out/per_step_summary.txt ;;
pmc)
  bash tools/profile_round.sh $out > $out/profile_round.log 2>&1 || exit $?
  tail -3 $out/profile_round.log ;;
sizes)
  timeout -k 10 200 python -u bench.py --n 2048 --warmup 5 --steps 20 --no-cpu > $out/n2048.log 2>&1 || exit $?
  line n2048 $out/n2048.log
  timeout -k 10 300 python -u bench.py --n 8192 --warmup 5 --steps 10 --no-cpu > $out/n8192.log 2>&1 || exit $?
  line n8192 $out/n8192.log
  timeout -k 10 400 python -u bench.py --n 16384 --warmup 3 --steps 4 --no-cpu > $out/n16384.log 2>&1 || exit $?
  line n16384 $out/n16384.log ;;
projection)
  timeout -k 10 600 python3 -u tools/slab_projection.py --n 4096 --ranks 1,2,4,8 > $out/projection_4096.log 2>&1 || exit $?
  tail -1 $out/projection_4096.log
  timeout -k 10 600 python3 -u tools/slab_projection.py --n 8192 --ranks 1,2,4,8 > $out/projection_8192.log 2>&1 || exit $?
  tail -1 $out/projection_8192.log
  timeout -k 10 900 python3 -u tools/slab_projection.py --weak-rows 2048 --ny 8192 --warmup 3 --steps 5 \
    > $out/projection_weak.log 2>&1 || exit $?
  tail -1 $out/projection_weak.log ;;
devflow)
  for w in 5 10 2000; do
    timeout -k 10 200 python -u bench.py --no-cpu --warmup $w --steps 40 --time-every 0 > $out/bench_w$w.log 2>&1 || exit $?
    line "warmup_$w" $out/bench_w$w.log
  done ;;
jacobi)
  timeout -k 10 300 python3 -u tools/sweep_c5.py --n 4096 8192 16384 > $out/sweeps.log 2>&1 || exit $?
  cat $out/sweeps.log ;;
fallbacks)
  # (r6) the grids the direct solve does not take: bench lines (MLUPS, step and kernel
  # rooflines) and kernel traces of the stretched cavity (ratio 1.0005 both ways / x only), a 4000^2 cavity
  # (ny not a power of two), the 2-rank host-transport channel, and the masked L-shape / step at 4096
  trace() {   # trace <name> <steps> <bench args...>: a kernel trace of the same command, per-step summary
    local nm=$1 st=$2; shift 2
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_$nm -o run -- \
      python3 "$@" > $out/trace_$nm.log 2>&1 || return $?
    python3 tools/trace_summary.py $(find $out/trace_$nm -name "*kernel_trace.csv" | head -1) $st > $out/${nm}_summary.txt
    head -14 $out/${nm}_summary.txt
  }
  for c in stretched xstretched; do
    timeout -k 10 300 python -u bench.py --case $c --warmup 5 --steps 20 > $out/$c.log 2>&1 || exit $?
    line $c $out/$c.log
    trace $c 25 bench.py --case $c --warmup 5 --steps 20 --no-cpu || exit $?
  done
  timeout -k 10 300 python -u bench.py --n 4000 --warmup 5 --steps 20 > $out/n4000.log 2>&1 || exit $?
  line n4000 $out/n4000.log
  trace n4000 25 bench.py --n 4000 --warmup 5 --steps 20 --no-cpu || exit $?
  timeout -k 10 400 python -u bench.py --case channel --gpus 2 --transport host --warmup 3 --steps 10 \
    > $out/channel_host2.log 2>&1 || exit $?
  line channel_host2 $out/channel_host2.log
  timeout -k 10 400 python -u tools/bench_bcs.py 4096 1024 4096 > $out/bcs_4096.log 2>&1 || exit $?
  cat $out/bcs_4096.log
  trace lshape_4096 5 tools/bench_bcs.py --lshape-only 4096 || exit $? ;;
*)
  echo "usage: bash tools/evidence.sh suite|bench|pmc|sizes|projection|devflow|jacobi|fallbacks [outdir]"; exit 2 ;;
esac
echo done
