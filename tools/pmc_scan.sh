# SQ / LDS PMC passes over the global scan (tools/microbench.py scan): tools/pmc_scan.sh -> gpurun_out/r05sc/{pa,pb}
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r05sc; mkdir -p $O; export TMPDIR=/tmp
MB="python3 $GRAFT_REPO_ROOT/tools/microbench.py scan --reps 2"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU --kernel-include-regex "k_scan_split" --output-format csv -d $O/pa -o run -- $MB > $O/pa.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex "k_scan_split" --output-format csv -d $O/pb -o run -- $MB > $O/pb.log 2>&1
