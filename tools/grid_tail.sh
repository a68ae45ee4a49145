#!/bin/bash
# Per-image phase time at grid sizes around whole rounds of resident
# workgroups (12 288 = 16 x 768, 13 056 = 17 x 768): tools/grid_tail.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
for n in 12288 12500 13056 12288 12500 13056; do
  timeout -k 10 120 python -u $R/tools/microbench.py local --ru 24 --images $n --ypair 1 --spread 3 --reps 5 | tail -1 >> $O/tail.jsonl
done
