#!/bin/bash
# A/B library from the current objects with some sources rebuilt under extra
# defines: tools/build_define.sh NAME a.hip[,b.hip] -DFOO=1 ... -> thunder_amd/ab/lib_NAME.so
set -e
R=$(cd $(dirname $0)/.. && pwd)
name=$1; src=$2; shift 2
T=$(mktemp -d /tmp/thxdef.XXXX)
objs=()
for o in $R/build/obj/*.o; do
  b=$(basename $o .o)
  if [[ ",$src," == *",$b.hip,"* ]]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics "$@" \
        -I$R/include -c $R/thunder_amd/csrc/$b.hip -o $T/$b.o
    objs+=($T/$b.o)
  else
    objs+=($o)
  fi
done
mkdir -p $R/thunder_amd/ab
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 ${objs[@]} -L/opt/rocm/lib \
    -Wl,-rpath,/opt/rocm/lib -lrccl -lhipfft -o $R/thunder_amd/ab/lib_$name.so
rm -rf $T
