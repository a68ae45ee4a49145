#!/bin/bash
# PF group-size A/B: pf_bench per library, then the bench step (tools/ab_lib.sh)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pfab
mkdir -p $O
cd $R
for L in default lib_pf32.so lib_pf64.so; do
  if [ "$L" = default ]; then unset THX_LIB; else export THX_LIB=$R/thunder_amd/ab/$L; fi
  echo "== $L" >> $O/pf.jsonl
  timeout -k 10 120 python tools/pf_bench.py >> $O/pf.jsonl 2>> $O/pf.err
done
unset THX_LIB
bash tools/ab_lib.sh pfab default lib_pf32.so lib_pf64.so
