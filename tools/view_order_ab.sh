#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab; mkdir -p $O
for k in 1 2; do for v in 1 0; do
  THX_VIEW_ORDER=$v timeout -k 10 300 python -u $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $O/r04vo3_$v.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('$O/r04vo3_$v.json').read().strip().splitlines()[-1]); print(json.dumps({'view_order': $v, 'value': d['value'], 'phases': d['roofline']['launch_ms_by_phase']}))" >> $O/r04vo3.jsonl
done; done
