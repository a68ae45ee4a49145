#!/bin/bash
# A/B of the local-phase kernel on the bench's own clouds (tools/data/clouds_r03.npz):
# the in-tree library vs thunder_amd/ab/lib_*.so (lib_count: wave-step counts).
# usage: tools/ab_clouds.sh TAG "phases" [extra microbench args]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for k in $2; do
  for L in "" $R/thunder_amd/ab/*.so; do
    extra=""
    case "$L" in *lib_count.so) extra="--counts 1 --reps 1";; esac
    THX_LIB=${L:-$R/thunder_amd/libthunder_amd.so} timeout -k 10 120 python tools/microbench.py local \
        --clouds ${CLOUDS:-tools/data/clouds_r03.npz} --k $k ${@:3} $extra \
        | sed "s|^{|{\"lib\": \"$(basename ${L:-new})\", |" >> $O/ab.jsonl
    tail -1 $O/ab.jsonl
  done
done
