#!/bin/bash
# Diagnostic builds of the library with extra -D flags into thunder_amd/ab/
# (A/B microbenchmarks only).  usage: tools/build_variants.sh NAME "-DFLAG ..." ...
set -e
R=$(cd $(dirname $0)/.. && pwd)
mkdir -p $R/thunder_amd/ab $R/build/var
while [ $# -gt 1 ]; do
  name=$1; flags=$2; shift 2
  objs=()
  for s in $R/thunder_amd/csrc/*.hip; do
    o=$R/build/var/${name}_$(basename ${s%.hip}).o
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics $flags -c $s -o $o &
    objs+=($o)
  done
  wait
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 ${objs[@]} -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrccl -lhipfft -o $R/thunder_amd/ab/lib_$name.so
done
