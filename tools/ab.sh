#!/bin/bash
# The one A/B driver: the headline bench (3 steps, no extras) once per library,
# in the order given, appending one JSON line per run (images/s, ms/step, the
# dominant kernel's per-phase times) to gpurun_out/ab/TAG.jsonl.
#   tools/ab.sh TAG NAME ...      NAME = prod (thunder_amd/libthunder_amd.so) or
#                                 the NAME of thunder_amd/ab/lib_NAME.so
# Variant libraries come from tools/build_define.sh NAME src.hip -DFOO=1 ...
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
O=$R/gpurun_out/ab
mkdir -p $O
for t in "$@"; do
  lib=$R/thunder_amd/ab/lib_$t.so
  [ $t = prod ] && lib=$R/thunder_amd/libthunder_amd.so
  THX_LIB=$lib timeout -k 10 300 python -u $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline \
      --no-extras > $O/${tag}_$t.json 2> $O/${tag}_$t.err
  python3 -c "import json; d=json.loads(open('$O/${tag}_$t.json').read().strip().splitlines()[-1]); print(json.dumps({'tag': '$t', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'phases': d['roofline']['launch_ms_by_phase']}))" >> $O/$tag.jsonl
done
