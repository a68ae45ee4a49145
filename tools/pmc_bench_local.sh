#!/bin/bash
# One PMC pass over the bench's k_local_fused dispatches (10 phases of one
# step): TA / TCP / TCC / SQ counters per phase.  GPU box, repo root:
#   tools/pmc_bench_local.sh OUTDIR
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex "k_local_fused" --output-format csv \
    -d $O/p -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extras \
    > $O/p.log 2>&1
