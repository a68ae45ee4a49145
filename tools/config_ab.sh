#!/bin/bash
# tools/config_bench.py per library, interleaved: tools/config_ab.sh TAG CONFIGS ROUNDS NAME ...
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; cfg=$2; rounds=$3; shift 3
O=$R/gpurun_out/ab; mkdir -p $O
for k in $(seq $rounds); do for t in "$@"; do
  lib=$R/thunder_amd/ab/lib_$t.so; [ $t = prod ] && lib=$R/thunder_amd/libthunder_amd.so
  THX_LIB=$lib timeout -k 10 300 python -u $R/tools/config_bench.py --only $cfg | while read -r line; do
    echo "{\"tag\": \"$t\", \"round\": $k, \"run\": $line}" >> $O/${tag}_config.jsonl; done
done; done
