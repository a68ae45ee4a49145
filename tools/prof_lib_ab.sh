#!/bin/bash
# rocprofv3 kernel stats of one command per library: tools/prof_lib_ab.sh TAG "CMD" NAME ...
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; cmd=$2; shift 2
export TMPDIR=/tmp
mkdir -p $R/gpurun_out/$tag
for t in "$@"; do
  lib=$R/thunder_amd/ab/lib_$t.so; [ $t = prod ] && lib=$R/thunder_amd/libthunder_amd.so
  (cd /tmp && THX_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $R/gpurun_out/$tag/$t -o run -- $cmd > $R/gpurun_out/$tag/$t.log 2>&1)
done
