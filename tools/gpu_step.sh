#!/bin/bash
# Run GPU steps in order; each: "SECONDS LOGNAME CMD...".  A step that fails
# with pytest's test-failure status (1) lets the next run; any other failure
# (fault, abort, time limit) ends the script there.
#   tools/gpu_step.sh TAG 'secs|name|cmd' ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
O=$R/gpurun_out/$tag
mkdir -p $O
export TMPDIR=/tmp
for step in "$@"; do
  secs=${step%%|*}; rest=${step#*|}; name=${rest%%|*}; cmd=${rest#*|}
  (cd $R && timeout -k 10 $secs bash -c "$cmd" > $O/$name.log 2>&1)
  rc=$?
  echo "$name rc=$rc" >> $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
