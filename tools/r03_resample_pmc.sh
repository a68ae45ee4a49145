#!/bin/bash
# HBM bytes of the k_pf_resample launches (one bench step): FETCH_SIZE and
# WRITE_SIZE in separate passes, plus the kernel trace for durations
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/rspmc
mkdir -p $O
export TMPDIR=/tmp
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv \
      --kernel-include-regex "k_pf_resample" -d $O/pmc$i -o run -- python3 $R/bench.py --steps 1 \
      --warmup 0 --no-cpu-baseline --no-extras > $O/pmc$i.log 2>&1)
done
