# SQ / TA PMC passes over the bench's k_local_fused launches: tools/pmc_local.sh TAG -> gpurun_out/TAG/{pa,pb}
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O; export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-extras --no-cpu-baseline"
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_VMEM_RD --kernel-include-regex "k_local_fused" --output-format csv -d $O/pa -o run -- $B > $O/pa.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU --kernel-include-regex "k_local_fused" --output-format csv -d $O/pb -o run -- $B > $O/pb.log 2>&1
