#!/bin/bash
# The product scan with and without its cancellation guard (no dvp dump in
# either since round 6): tools/scan_guard_ab.sh TAG ROUNDS
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab; mkdir -p $O
for k in $(seq $2); do
  for g in default 0; do
    arg=""; [ $g = 0 ] && arg="--guard 0"
    run=$(timeout -k 10 120 python -u $R/tools/microbench.py scan $arg | tail -1)
    echo "{\"guard\": \"$g\", \"round\": $k, \"run\": $run}" >> $O/$1_guard.jsonl
  done
done
