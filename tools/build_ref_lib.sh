#!/bin/bash
# A/B library from a git revision's sources: tools/build_ref_lib.sh REF NAME
#   -> thunder_amd/ab/lib_NAME.so (all of thunder_amd/csrc + include at REF)
set -e
R=$(cd $(dirname $0)/.. && pwd)
ref=$1; name=$2
T=$(mktemp -d /tmp/thxref.XXXX)
mkdir -p $T/src/thunder_amd $T/obj
git -C $R archive $ref thunder_amd/csrc include | tar -x -C $T/src
pids=()
for f in $T/src/thunder_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics \
      -I$T/src/include -c $f -o $T/obj/$(basename $f .hip).o &
  pids+=($!)
done
for p in ${pids[@]}; do wait $p; done
mkdir -p $R/thunder_amd/ab
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $T/obj/*.o -L/opt/rocm/lib \
    -Wl,-rpath,/opt/rocm/lib -lrccl -lhipfft -o $R/thunder_amd/ab/lib_$name.so
rm -rf $T
