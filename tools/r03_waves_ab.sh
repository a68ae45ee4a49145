#!/bin/bash
# A/B of the pair-form y-pair kernel's occupancy / pipelining: waves per SIMD
# (THX_NOBOX_WAVES 4 / 6 / 8) and patches per barrier pair (THX_NOBOX_PP 1 / 2)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${AB_TAG:-waves}
mkdir -p $O
run() {
  tag=$1; lib=$2
  THX_LIB=$R/$lib timeout -k 10 300 python -u $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline \
      --no-extras > $O/$tag.json 2> $O/$tag.err
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print(json.dumps({'tag': '$tag', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'phases': d['roofline']['launch_ms_by_phase']}))" >> $O/ab.jsonl
}
run def thunder_amd/libthunder_amd.so
run nt thunder_amd/ab/lib_nt.so
run def_b thunder_amd/libthunder_amd.so
run nt_b thunder_amd/ab/lib_nt.so
