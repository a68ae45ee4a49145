#!/bin/bash
# TCP / TCC counters of the gather probes (tools/probes/l2_roof.hip), to put
# the local phase's PMC counts and the probes' rates in the same units.
#   tools/pmc_probe.sh OUTDIR [table_MB ...]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1; shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for mb in ${@:-0.016 2}; do
  timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE \
      --output-format csv -d $O/mb$mb -o run -- $R/tools/probes/l2_roof_bin $mb > $O/mb$mb.log 2>&1
done
