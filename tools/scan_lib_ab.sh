#!/bin/bash
# Scan microbench (default guard) per library, interleaved:
#   tools/scan_lib_ab.sh TAG ROUNDS NAME ...   (prod = the in-tree library)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; rounds=$2; shift 2
O=$R/gpurun_out/ab; mkdir -p $O
for k in $(seq $rounds); do for t in "$@"; do
  lib=$R/thunder_amd/ab/lib_$t.so; [ $t = prod ] && lib=$R/thunder_amd/libthunder_amd.so
  run=$(THX_LIB=$lib timeout -k 10 120 python -u $R/tools/microbench.py scan | tail -1)
  echo "{\"tag\": \"$t\", \"round\": $k, \"run\": $run}" >> $O/${tag}_scan.jsonl
done; done
