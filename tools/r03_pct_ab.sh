#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pct
mkdir -p $O
for pct in 20 25 20 25; do
  THX_YPAIR_MAX_PCT=$pct timeout -k 10 300 python -u $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline \
      --no-extras > $O/p$pct.json 2> $O/p$pct.err
  python3 -c "import json; d=json.loads(open('$O/p$pct.json').read().strip().splitlines()[-1]); print(json.dumps({'pct': $pct, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'phases': d['roofline']['launch_ms_by_phase']}))" >> $O/ab.jsonl
done
