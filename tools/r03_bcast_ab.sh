#!/bin/bash
# A/B: the quad-cooperative kernels computing each sample's cell once per quad
# (DPP broadcast; libthunder_amd.so) against the previous build (lib_prev.so).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/bcast
mkdir -p $O
(cd $R && timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q \
    --timeout 120 --timeout-method thread > $O/tests.log 2>&1)
run() {
  tag=$1; lib=$2
  THX_LIB=$R/thunder_amd/$lib timeout -k 10 300 python -u $R/bench.py --steps 3 --warmup 1 \
      --no-cpu-baseline --no-extras > $O/$tag.json 2> $O/$tag.err
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print(json.dumps({'tag': '$tag', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'pose_err': d['median_pose_error_deg'], 'phases': d['roofline']['launch_ms_by_phase']}))" >> $O/ab.jsonl
}
run prev lib_prev.so
run bcast libthunder_amd.so
run prev_b lib_prev.so
run bcast_b libthunder_amd.so
