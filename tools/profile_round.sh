#!/bin/bash
# Kernel trace + HBM PMC passes of the bench workload (run on the GPU box from the repo root):
#   bash tools/profile_round.sh <outdir under gpurun_out/>
# writes <outdir>/trace (kernel trace + stats), <outdir>/fetch, <outdir>/write (PMC),
# <outdir>/per_step_summary.txt and <outdir>/pmc_traffic.json (per-kernel HBM bytes; copy it to
# profiles/pmc_traffic.json, which bench.py reads for each kernel's roofline.traffic).  Each
# rocprofv3 run is its own pass (--pmc never combined with the runtime/sys trace domains).
set -e
out=${1:-gpurun_out/prof}
export TMPDIR=/tmp
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu > $out/trace.log 2>&1
python3 tools/trace_summary.py $(find $out/trace -name "*kernel_trace.csv" | head -1) 13 > $out/per_step_summary.txt
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $out/fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $out/write.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $out/valu -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $out/valu.log 2>&1
python3 tools/pmc_summarize.py 4096 $out/fetch $out/write $out/pmc_traffic.json \
  'restrict=k_sweep2<0, false, 1=26' 'prolong=k_sweep2<0, (true|false), 2=26' 'cycle=k_sweep4=28' \
  'jacobi_sweep=k_jacobi_s<double=24' 'jacobi_sweep_fp32=k_jacobi_s<float=12' \
  'helmholtz=k_sweep3<(0|3), true=48' 'rhs=k_rhs_s<=64' 'rhs_sc=k_rhs_sc<=88' 'band=k_helm_band=5.8125' \
  'k5=k_cell_s<(5|6)>=40' 'k3=k_cell_s<3>=24' \
  'fps_dct=k_fps_dct<=16' 'fps_dct_div=k_fps_dct_div(_r)?<=24' 'fps_idct=k_fps_idct(_r)?<=16' 'fps_t1b=k_fps_t1b=8' 'fps_t2b=k_fps_t2b=16' 'fps_mid=k_fps_mid=0.5'
# (one rank's Helmholtz residual pass is the two-field launch k_sweep3<FUSE_UV = 3>: 2 x 24 B/cell; the
# bench's helmholtz roofline is per component, so the entry is halved)
python3 - $out/pmc_traffic.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); h = d["kernels"].get("helmholtz")
if h:
    for k in ("fetch_bytes_corrected", "write_bytes", "kernel_bytes_per_launch", "algorithmic_bytes_per_launch"):
        h[k] = h[k] / 2 if h.get(k) is not None else None
    h["note"] = "per velocity component: the two-field launch's bytes / 2"
json.dump(d, open(sys.argv[1], "w"), indent=1)
PY
python3 tools/pmc_summarize.py --valu 4096 $out/valu $out/valu_per_cell.json 'rhs=k_rhs_s<' 'helmholtz=k_sweep3<(0|3), true' \
  'restrict=k_sweep2<0, false, 1' 'prolong=k_sweep2<0, (true|false), 2' 'cycle=k_sweep4' 'k5=k_cell_s<(5|6)>' 'k3=k_cell_s<3>' \
  'fps_dct=k_fps_dct<' 'fps_dct_div=k_fps_dct_div(_r)?<' 'fps_idct=k_fps_idct(_r)?<' 'fps_t1b=k_fps_t1b' 'fps_t2b=k_fps_t2b' 'fps_mid=k_fps_mid'
