#!/bin/bash
# Sub-batch concurrency A/B: the headline bench (3 steps, no extras) with the
# batch as concurrent sub-batches on HIP streams (bench.py --streams / --chunk),
# one JSON line per run to gpurun_out/ab/TAG_streams.jsonl.
#   tools/streams_ab.sh TAG "ARGS" ...      ("" = one stream, the whole batch)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
O=$R/gpurun_out/ab
mkdir -p $O
for args in "$@"; do
  timeout -k 10 300 python -u $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras $args \
      > $O/${tag}_streams.json 2> $O/${tag}_streams.err
  python3 -c "import json; d=json.loads(open('$O/${tag}_streams.json').read().strip().splitlines()[-1]); print(json.dumps({'args': '$args', 'value': d['value'], 'ms_per_step': d['ms_per_step']}))" >> $O/${tag}_streams.jsonl
done
