#!/bin/bash
# A/B of library builds on the bench (GPU box): tools/ab_lib.sh TAG lib_a.so lib_b.so ...
# (THX_LIB selects the library; "default" = thunder_amd/libthunder_amd.so)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; shift
mkdir -p $O
i=0
for L in "$@"; do
  i=$((i+1))
  if [ "$L" = default ]; then unset THX_LIB; else export THX_LIB=$R/thunder_amd/ab/$L; fi
  (cd $R && timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-extras --no-cpu-baseline > $O/ab$i.json 2> $O/ab$i.err)
  echo "$L" >> $O/ab$i.json
done
