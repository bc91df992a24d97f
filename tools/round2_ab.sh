#!/bin/bash
# RCCL loopback / virtual-slab tests, the 8192^2 slab projection, then an A/B of library builds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py -v -p no:cacheprovider --timeout=120 --timeout-method=thread > gpurun_out/pytest_rccl.log 2>&1
rc=$?; echo "rccl pytest rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/pytest_rccl.log | tail -12
[ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python -u tools/slab_projection.py > gpurun_out/projection.log 2>&1
rc=$?; echo "projection rc=$rc"; grep -v "version\|Hostname\|Librccl" gpurun_out/projection.log
[ $rc -ne 0 ] && exit $rc
[ -n "$AB_LIBS" ] && bash tools/ab_lib.sh $AB_LIBS
