#!/bin/bash
# Quick GPU iteration: selected parity tests + local / scan microbench.
# usage: tools/gpu_iter.sh TAG "pytest -k expr" "microbench arg sets separated by ;"
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
if [ -n "$2" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$2" > $O/tests.log 2>&1
fi
IFS=';' read -ra SETS <<< "$3"
for a in "${SETS[@]}"; do
  timeout -k 10 120 python tools/microbench.py $a >> $O/mb.jsonl 2>> $O/mb.err
done
