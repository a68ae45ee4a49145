#!/bin/bash
# The product scan with and without its cancellation guard (no dvp dump in
# either since round 6): tools/scan_guard_ab.sh TAG ROUNDS
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab; mkdir -p $O
for k in $(seq $2); do
  for g in 1 0; do
    run=$(timeout -k 10 120 python -u $R/tools/microbench.py scan --guard $g | tail -1)
    echo "{\"guard\": $g, \"round\": $k, \"run\": $run}" >> $O/$1_guard.jsonl
  done
done
