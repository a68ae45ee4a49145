#!/bin/bash
# A/B variant of one source: tools/ab_build.sh NAME SRC "-DFLAG ..." -> ab_so/NAME.so (travels to the GPU box; git-ignored)
set -e
name=$1; src=$2; flags=$3
R=$(cd $(dirname $0)/.. && pwd)
mkdir -p $R/build/ab $R/ab_so
srcpath=$src; [ -f "$srcpath" ] || srcpath=$R/thunder_amd/csrc/$src
base=${4:-$(basename $src .hip)}
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics $flags -I$R/thunder_amd/csrc -c $srcpath -o $R/build/ab/$name.o
objs=$(ls $R/build/obj/*.o | grep -v "/$base.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs $R/build/ab/$name.o -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrccl -lhipfft -o $R/ab_so/$name.so
