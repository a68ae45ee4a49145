#!/bin/bash
# L1 / L2 / TA counters of k_local_fused on the bench's evaluated clouds
# (tools/data/clouds_eval.npz) for the half-complex and bricked layouts.
# usage (GPU box, repo root): tools/pmc_gather.sh OUTDIR "phases" [lib]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
for k in $2; do for br in 0 1; do
  tag=k${k}_b${br}
  THX_LIB=${3:-$R/thunder_amd/libthunder_amd.so} timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "k_local_fused" \
      --output-format csv -d $O/$tag -o run -- python3 $R/tools/microbench.py local \
      --clouds $R/tools/data/clouds_eval.npz --k $k --images 4096 --reps 2 --bricks $br > $O/$tag.log 2>&1
done; done
