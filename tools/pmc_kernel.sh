#!/bin/bash
# PMC passes over one microbench kernel (run on the GPU box from the repo root).
# usage: tools/pmc_kernel.sh OUTDIR KERNEL_REGEX microbench-args...
set -e
out=$1; shift
rx=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/$out
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES"
P3="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $P --kernel-include-regex "$rx" --output-format csv \
      -d $R/$out/p$i -o run -- python3 $R/tools/microbench.py "$@" --reps 2 > $R/$out/p$i.log 2>&1
done
