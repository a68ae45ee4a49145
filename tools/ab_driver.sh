#!/bin/bash
# A/B of driver options on the bench (run on the GPU box): tools/ab_driver.sh TAG "args1" "args2" ...
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; shift
mkdir -p $O
i=0
for a in "$@"; do
  i=$((i+1))
  (cd $R && timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-extras --no-cpu-baseline $a > $O/ab$i.json 2> $O/ab$i.err)
  echo "$a" >> $O/ab$i.json
done
