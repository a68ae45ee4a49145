#!/bin/bash
# Kernel-trace A/B of the bench: the in-tree library vs thunder_amd/ab/*.so.
# usage: tools/ab_prof.sh TAG [bench args]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
for L in "" $R/thunder_amd/ab/*.so; do
  n=$(basename ${L:-new} .so)
  (cd /tmp && THX_LIB=${L:-$R/thunder_amd/libthunder_amd.so} timeout -k 10 200 rocprofv3 \
      --kernel-trace --stats --output-format csv -d $O/$n -o run -- python3 $R/bench.py \
      --steps 1 --warmup 0 --no-cpu-baseline --no-extras ${@:2} > $O/$n.json 2> $O/$n.err)
done
