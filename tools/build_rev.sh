#!/bin/bash
# A/B library from the current sources with some files taken from a git
# revision: tools/build_rev.sh NAME REV path/in/repo ... -> thunder_amd/ab/lib_NAME.so
set -e
R=$(cd $(dirname $0)/.. && pwd)
name=$1; rev=$2; shift 2
T=$(mktemp -d /tmp/thxrev.XXXX)
mkdir -p $T/src/thunder_amd $T/obj
cp -r $R/include $T/src/
cp -r $R/thunder_amd/csrc $T/src/thunder_amd/
for f in "$@"; do git -C $R show $rev:$f > $T/src/$f; done
objs=()
for s in $T/src/thunder_amd/csrc/*.hip; do
  o=$T/obj/$(basename ${s%.hip}).o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -c $s -o $o &
  objs+=($o)
done
wait
mkdir -p $R/thunder_amd/ab
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 ${objs[@]} -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrccl -lhipfft -o $R/thunder_amd/ab/lib_$name.so
rm -rf $T
