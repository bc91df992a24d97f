set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
o=gpurun_out/r06e
mkdir -p $o
timeout -k 10 120 python -u tools/k1_timing_probe.py > $o/probe_plain.log 2>&1 || exit 1
cat $o/probe_plain.log
NSGPU_EXT_TIMING=0 timeout -k 10 120 python -u tools/k1_timing_probe.py > $o/probe_marker.log 2>&1 || exit 1
cat $o/probe_marker.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace -o run -- python3 tools/k1_timing_probe.py > $o/probe_rocprof.log 2>&1 || exit 1
cat $o/probe_rocprof.log
grep -E "k_rhs" $o/trace/run_kernel_stats.csv | cut -d, -f1-4
timeout -k 10 100 ./tools/membw2 copy > $o/membw_copy.log 2>&1 || exit 1
cat $o/membw_copy.log
timeout -k 10 100 ./tools/membw2 k1c > $o/membw_k1c.log 2>&1 || exit 1
cat $o/membw_k1c.log
timeout -k 10 100 ./tools/membw2 k1 > $o/membw_k1.log 2>&1 || exit 1
cat $o/membw_k1.log
