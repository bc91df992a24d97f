#!/bin/bash
# One gpurun call: GPU parity tests, a short bench, a rocprofv3 kernel-trace of the bench.
# Stops at the first crash-type exit (abort / segfault / timeout); a plain test failure
# (pytest exit 1) still lets the bench run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fault() { case $1 in 0|1) return 1;; *) return 0;; esac; }
PYTEST_ARGS=${PYTEST_ARGS:-"tests -m gpu -v"}
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest $PYTEST_ARGS -p no:cacheprovider --timeout=${TEST_TIMEOUT:-300} --timeout-method=thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log
if fault $rc; then exit $rc; fi
[ -n "$SKIP_BENCH" ] && exit 0
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:---steps 3 --warmup 1} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
if fault $rc || [ $rc -ne 0 ]; then exit $rc; fi
[ -n "$SKIP_PROF" ] && exit 0
timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py ${PROF_ARGS:---steps 2 --warmup 1 --no-cpu} > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
