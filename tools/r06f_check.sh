# round-6 check: the whole GPU suite, the driver-form bench, and the fallback evidence.
#   gpurun -- bash tools/r06f_check.sh [outdir]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
o=${1:-gpurun_out/r06f}
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout=300 --timeout-method=thread \
  > $o/tests.log 2>&1
rc=$?
tail -3 $o/tests.log; grep -E "^FAILED" $o/tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 > $o/bench_driver_form.log 2>&1 || exit 1
python3 tools/bench_line.py driver_form $o/bench_driver_form.log
bash tools/evidence.sh fallbacks $o/fb > $o/fallbacks.log 2>&1 || { tail -20 $o/fallbacks.log; exit 1; }
grep -vE "^nsg|^__amd|total GPU" $o/fallbacks.log
timeout -k 10 120 ./tools/membw2 strip > $o/membw_strip.log 2>&1 || exit 1
cat $o/membw_strip.log
