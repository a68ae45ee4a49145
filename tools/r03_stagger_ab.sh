#!/bin/bash
# A/B of staggered sub-batches (bench.py --stagger): one stream vs 2-3
# streams, the scan of sub-batch c beside the phases of c-1.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/stagger
mkdir -p $O
run() {
  tag=$1; shift
  timeout -k 10 300 python -u $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras "$@" \
      > $O/$tag.json 2> $O/$tag.err
  python3 -c "import json,sys; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print(json.dumps({'tag': '$tag', 'args': sys.argv[1:], 'value': d['value'], 'ms_per_step': d['ms_per_step']}))" "$@" >> $O/ab.jsonl
}
run one
run s2c6250 --streams 2 --chunk 6250
run s2c6250st --streams 2 --chunk 6250 --stagger 1
run s2c3125st --streams 2 --chunk 3125 --stagger 1
run s3c4167st --streams 3 --chunk 4167 --stagger 1
run one_b
