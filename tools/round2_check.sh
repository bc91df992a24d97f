#!/bin/bash
# GPU session of round 2: RCCL loopback tests first (new call sites), the full GPU suite,
# the default bench and the 8192^2 slab projection.  Stops at the first crash-type exit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fault() { case $1 in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py -v -p no:cacheprovider --timeout=120 --timeout-method=thread > gpurun_out/pytest_rccl.log 2>&1
rc=$?; echo "rccl pytest rc=$rc"; tail -15 gpurun_out/pytest_rccl.log
if fault $rc; then exit $rc; fi
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout=300 --timeout-method=thread --deselect tests/test_gpu_rccl.py > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -15
if fault $rc; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench.log
if fault $rc; then exit $rc; fi
timeout -k 10 300 python -u tools/slab_projection.py > gpurun_out/projection.log 2>&1
rc=$?; echo "projection rc=$rc"; cat gpurun_out/projection.log
exit $rc
