set -e
R=$GRAFT_REPO_ROOT
bash $R/tools/pmc_kernel.sh gpurun_out/r01s2c/pmc k_scan_bf16x3 scan
