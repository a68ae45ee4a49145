#!/bin/bash
# A/B of the run-length inferACG (k_pf_mean / calVari / balanceWeight):
# fixed-point iterations and k_pf_mean time on the bench's clouds, then the
# bench step, against thunder_amd/ab/lib_acgold.so (the strided version)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${AB_TAG:-acg}
OLD=${OLD_LIB:-thunder_amd/ab/lib_acgold.so}
mkdir -p $O
THX_LIB=$R/thunder_amd/libthunder_amd.so timeout -k 10 300 python -u $R/tools/pf_iters.py > $O/iters_new.jsonl
THX_LIB=$R/$OLD timeout -k 10 300 python -u $R/tools/pf_iters.py > $O/iters_old.jsonl
run() {
  tag=$1; lib=$2
  THX_LIB=$R/$lib timeout -k 10 300 python -u $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline \
      --no-extras > $O/$tag.json 2> $O/$tag.err
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print(json.dumps({'tag': '$tag', 'value': d['value'], 'ms_per_step': d['ms_per_step']}))" >> $O/ab.jsonl
}
run new thunder_amd/libthunder_amd.so
run old $OLD
run new_b thunder_amd/libthunder_amd.so
run old_b $OLD
