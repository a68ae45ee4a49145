#!/bin/bash
# Compact-ball placement A/B: the headline bench (3 steps, no extras) per
# THX_YPAIR_OFFSET value ("-" = unset: the ball right after the buffers before
# it), interleaved over ROUNDS, one JSON line each to gpurun_out/ab/TAG.jsonl.
#   tools/ball_offset_ab.sh TAG ROUNDS OFFSET ...
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; rounds=$2; shift 2
O=$R/gpurun_out/ab
mkdir -p $O
for k in $(seq $rounds); do
  for off in "$@"; do
    if [ "$off" = "-" ]; then unset THX_YPAIR_OFFSET; else export THX_YPAIR_OFFSET=$off; fi
    timeout -k 10 300 python -u $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras \
        > $O/${tag}_run.json 2> $O/${tag}_run.err
    python3 -c "import json; d=json.loads(open('$O/${tag}_run.json').read().strip().splitlines()[-1]); print(json.dumps({'offset': '$off', 'round': $k, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'phases': d['roofline']['launch_ms_by_phase']}))" >> $O/$tag.jsonl
  done
done
