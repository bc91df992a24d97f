#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of the bench's finest passes for each library given:
#   bash tools/ab_pmc.sh lib1.so lib2.so ...   -> gpurun_out/ab_pmc/<k>/pmc_traffic.json
set -e
export TMPDIR=/tmp
k=0
for lib in "$@"; do
  k=$((k + 1)); out=gpurun_out/ab_pmc/$k
  mkdir -p $out
  NSGPU_LIB=$lib timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $out/fetch.log 2>&1
  NSGPU_LIB=$lib timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $out/write.log 2>&1
  python3 tools/pmc_summarize.py 4096 $out/fetch $out/write $out/pmc_traffic.json \
    'restrict=k_sweep2<0, false, 1=28' 'prolong=k_sweep2<0, (true|false), 2=26' 'helmholtz=k_sweep3<(0|3), true=48' > /dev/null
  python3 - "$lib" $out/pmc_traffic.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))["kernels"]
print(sys.argv[1], " ".join(f"{n}={v['kernel_bytes_per_launch'] / v['algorithmic_bytes_per_launch']:.3f}x"
                            for n, v in d.items() if v.get("kernel_bytes_per_launch")))
PY
done
