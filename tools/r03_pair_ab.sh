#!/bin/bash
# A/B of the route's wide-cloud kernel: quad y-pair (default) vs the pair form
# (THX_YPAIR_KERNEL=2) at the default threshold and on every phase.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pair
mkdir -p $O
(cd $R && timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 \
    --timeout-method thread > $O/parity.log 2>&1)
(cd $R && THX_YPAIR_KERNEL=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_driver.py -x -q \
    --timeout 120 --timeout-method thread > $O/driver.log 2>&1)
run() {
  tag=$1; k=$2; pct=$3
  THX_YPAIR_KERNEL=$k THX_YPAIR_MAX_PCT=$pct timeout -k 10 300 python -u $R/bench.py --steps 3 \
      --warmup 1 --no-cpu-baseline --no-extras > $O/$tag.json 2> $O/$tag.err
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print(json.dumps({'tag': '$tag', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'pose_err': d['median_pose_error_deg'], 'phases': d['roofline']['launch_ms_by_phase']}))" >> $O/ab.jsonl
}
run quad20 0 20
run pair20 2 20
run pair101 2 101
run quad20_b 0 20
run pair20_b 2 20
