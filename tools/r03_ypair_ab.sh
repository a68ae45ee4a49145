#!/bin/bash
# A/B of the phases' projectee layout in the driver: half-complex (routed
# staged / box-less) vs the y-pair copy (THX_PHASE_LAYOUT=ypair), each with
# and without the orientation-sorted XCD launch order (THX_XCD_ORDER=1).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ypair
mkdir -p $O
(cd $R && timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 \
    --timeout-method thread > $O/parity.log 2>&1)
run() {
  tag=$1; lay=$2; xo=$3; shift 3
  THX_PHASE_LAYOUT=$lay THX_XCD_ORDER=$xo timeout -k 10 300 python -u $R/bench.py --steps 3 \
      --warmup 1 --no-cpu-baseline --no-extras "$@" > $O/$tag.json 2> $O/$tag.err
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print(json.dumps({'tag': '$tag', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'pose_err': d['median_pose_error_deg'], 'phases': d['roofline']['launch_ms_by_phase']}))" >> $O/ab.jsonl
}
run ft ft 0
run ft_xo ft 1
run ypair ypair 0
run ypair_xo ypair 1
run ft_b ft 0
run ypair_xo_b ypair 1
