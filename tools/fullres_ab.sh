#!/bin/bash
# Full-resolution y-pair local phase (box 256, rU 126, 512 images) per cloud
# spread, libraries interleaved: tools/fullres_ab.sh TAG NAME ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
O=$R/gpurun_out/ab; mkdir -p $O
for k in 1 2; do for t in "$@"; do for sp in 1.5 2.0 3.0; do
  lib=$R/thunder_amd/ab/lib_$t.so; [ $t = prod ] && lib=$R/thunder_amd/libthunder_amd.so
  run=$(THX_LIB=$lib timeout -k 10 200 python -u $R/tools/microbench.py local --ru 126 --images 512 --ypair 1 --spread $sp --reps 3 | tail -1)
  echo "{\"tag\": \"$t\", \"spread\": $sp, \"run\": $run}" >> $O/${tag}_fullres.jsonl
done; done; done
