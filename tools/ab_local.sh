#!/bin/bash
# A/B of the local-phase kernel: the in-tree library vs thunder_amd/ab/*.so
# over particle-cloud spreads.  usage: tools/ab_local.sh TAG "spreads" [extra args]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for sp in $2; do
  for L in "" $R/thunder_amd/ab/*.so; do
    THX_LIB=${L:-$R/thunder_amd/libthunder_amd.so} timeout -k 10 120 python tools/microbench.py local \
        --spread $sp --reps 5 ${@:3} | sed "s|^{|{\"lib\": \"$(basename ${L:-new})\", \"spread\": $sp, |" >> $O/ab.jsonl
  done
done
