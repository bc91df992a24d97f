cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
bash tools/ab_lib.sh $(for L in ${PMC_LIBS:-fpnt1 fpnt0}; do echo abl/libnsgpu_$L.so; done) || exit 1
for L in ${PMC_LIBS:-fpnt1 fpnt0}; do
  NSGPU_LIB=abl/libnsgpu_$L.so timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_$L/fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > /dev/null 2>&1 || exit 1
  NSGPU_LIB=abl/libnsgpu_$L.so timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_$L/write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > /dev/null 2>&1 || exit 1
  python3 tools/pmc_summarize.py 4096 gpurun_out/pmc_$L/fetch gpurun_out/pmc_$L/write gpurun_out/pmc_$L/t.json 'prolong=k_sweep2<0, false, 2>=26' 'restrict=k_sweep2<0, false, 1>=28' > /dev/null
  python3 -c "
import json; d=json.load(open('gpurun_out/pmc_$L/t.json'))
print('$L', {k: round(v['kernel_bytes_per_launch']/v['algorithmic_bytes_per_launch'],3) for k,v in d['kernels'].items()})"
done
