#!/bin/bash
# A/B of the headline bench: the in-tree library vs thunder_amd/ab/*.so.
# usage: tools/ab_bench.sh TAG [bench args]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for L in "" $R/thunder_amd/ab/*.so; do
  n=$(basename ${L:-new})
  THX_LIB=${L:-$R/thunder_amd/libthunder_amd.so} timeout -k 10 300 python -u bench.py \
      --no-cpu-baseline ${@:2} > $O/bench_$n.json 2> $O/bench_$n.err
done
