#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pfab2
mkdir -p $O
cd $R
export THX_LIB=$R/thunder_amd/ab/lib_pf8.so
timeout -k 10 120 python tools/pf_bench.py >> $O/pf.jsonl 2>> $O/pf.err
unset THX_LIB
bash tools/ab_lib.sh pfab2 default lib_pf8.so
