#!/bin/bash
# build a libnsgpu.so variant with extra -D flags into abl/ (A/B with tools/ab_lib.sh):
#   bash tools/build_variant.sh abl/libnsgpu_x.so -DFOO=1 ...
set -e
out=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
cd "$root/navierstokessolver_amd/csrc"
make -s ns_solver.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -I../../include "$@" -c -o $tmp/k.o ns_kernels.hip
mkdir -p "$root/$(dirname $out)"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$root/$out" $tmp/k.o ns_solver.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf $tmp
