#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
for k in 1 2; do
for t in prod ec8 ec8w3; do
  lib=$R/thunder_amd/ab/lib_$t.so; [ $t = prod ] && lib=$R/thunder_amd/libthunder_amd.so
  THX_LIB=$lib timeout -k 10 120 python -u $R/tools/recon_time.py $t | tail -1
done; done
