#!/bin/bash
# A/B library from the current objects with ONE source rebuilt under extra
# defines: tools/build_define.sh NAME file.hip -DFOO=1 ... -> thunder_amd/ab/lib_NAME.so
set -e
R=$(cd $(dirname $0)/.. && pwd)
name=$1; src=$2; shift 2
T=$(mktemp -d /tmp/thxdef.XXXX)
objs=()
for o in $R/build/obj/*.o; do
  if [ "$(basename $o)" = "${src%.hip}.o" ]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics "$@" \
        -I$R/include -c $R/thunder_amd/csrc/$src -o $T/$(basename $o)
    objs+=($T/$(basename $o))
  else
    objs+=($o)
  fi
done
mkdir -p $R/thunder_amd/ab
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 ${objs[@]} -L/opt/rocm/lib \
    -Wl,-rpath,/opt/rocm/lib -lrccl -lhipfft -o $R/thunder_amd/ab/lib_$name.so
rm -rf $T
