#!/bin/bash
# kernel traces of the headline bench per library: tools/prof_ab.sh TAG NAME...
R=$GRAFT_REPO_ROOT; tag=$1; shift; O=$R/gpurun_out/$tag; mkdir -p $O; export TMPDIR=/tmp
for t in "$@"; do
  lib=$R/thunder_amd/ab/lib_$t.so; [ $t = prod ] && lib=$R/thunder_amd/libthunder_amd.so
  (cd /tmp && THX_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$t -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras > $O/prof_$t.json 2> $O/prof_$t.err) || exit 1
done
