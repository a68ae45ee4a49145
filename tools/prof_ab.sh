#!/bin/bash
# Kernel-time A/B of library builds on the bench (GPU box, repo root):
#   tools/prof_ab.sh TAG lib_a.so|default ...  -> gpurun_out/TAG/<lib>_kernel_stats.csv
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1; shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  if [ $L = default ]; then unset THX_LIB; else export THX_LIB=$R/thunder_amd/ab/$L; fi
  rm -rf /tmp/pfab
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pfab -o run -- \
      python3 $R/bench.py --steps 3 --warmup 1 --no-extras --no-cpu-baseline > $O/$L.log 2>&1
  cp $(find /tmp/pfab -name "*kernel_stats.csv" | head -1) $O/${L}_kernel_stats.csv
done
