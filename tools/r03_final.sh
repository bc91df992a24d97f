#!/bin/bash
# round-3 closing evidence: the default bench line and the driver's form (both with the CPU
# baseline leg), a kernel trace + stats of the driver's form, PMC traffic / VALU passes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${OUT:-r03_final}; mkdir -p $out
timeout -k 10 400 python -u bench.py > $out/bench_default.log 2>&1 || exit $?
python3 tools/bench_line.py default $out/bench_default.log
timeout -k 10 400 python -u bench.py --gpus 1 --warmup 5 --steps 20 > $out/bench_driver_form.log 2>&1 || exit $?
python3 tools/bench_line.py driver_form $out/bench_driver_form.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --warmup 5 --steps 20 --no-cpu > $out/trace.log 2>&1 || exit $?
python3 tools/trace_summary.py $(find $out/trace -name "*kernel_trace.csv" | head -1) 25 > $out/per_step_summary.txt
head -12 $out/per_step_summary.txt
bash tools/profile_round.sh $out/prof > $out/profile_round.log 2>&1 || exit $?
echo done
