#!/bin/bash
# FETCH_SIZE calibration on the GPU box: tools/calib/run_calib.sh OUTDIR
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 $R/tools/calib/fetch_calib > $O/calib_plain.txt 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/calib_fetch -o run -- $R/tools/calib/fetch_calib > $O/calib_fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $O/calib_req -o run -- $R/tools/calib/fetch_calib > $O/calib_req.log 2>&1
