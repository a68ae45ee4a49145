#!/bin/bash
# inferACG probe per library: tools/pf_probe_ab.sh TAG NAME ... -> gpurun_out/TAG/probe_NAME.log (+ dumps)
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
O=$R/gpurun_out/$tag; mkdir -p $O
for t in "$@"; do
  lib=$R/thunder_amd/ab/lib_$t.so; [ $t = prod ] && lib=$R/thunder_amd/libthunder_amd.so
  THX_LIB=$lib timeout -k 10 200 python -u $R/tools/pf_probe.py --dump $O/dump_$t > $O/probe_$t.log 2>&1 || exit $?
done
