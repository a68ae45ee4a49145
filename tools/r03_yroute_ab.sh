#!/bin/bash
# The device route with the y-pair kernel for wide clouds (default) against
# the route without it (THX_PHASE_LAYOUT=ft): GPU tests, then the bench twice each.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/yroute
mkdir -p $O
(cd $R && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 \
    --timeout-method thread > $O/tests.log 2>&1)
run() {
  tag=$1; lay=$2
  THX_PHASE_LAYOUT=$lay timeout -k 10 300 python -u $R/bench.py --steps 3 --warmup 1 \
      --no-cpu-baseline --no-extras > $O/$tag.json 2> $O/$tag.err
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print(json.dumps({'tag': '$tag', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'pose_err': d['median_pose_error_deg'], 'phases': d['roofline']['launch_ms_by_phase']}))" >> $O/ab.jsonl
}
run route_yp route
run ft ft
run route_yp_b route
run ft_b ft
