#!/bin/bash
# A/B of the resample CDF in LDS vs the global workspace: rocprof kernel
# stats of one bench step per library, then the bench step twice each
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/cdf
mkdir -p $O
export TMPDIR=/tmp
for v in new:thunder_amd/libthunder_amd.so old:thunder_amd/ab/lib_cdfglob.so; do
  tag=${v%%:*}; lib=${v#*:}
  (cd /tmp && THX_LIB=$R/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $O/prof_$tag -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline \
      --no-extras > $O/prof_$tag.json 2> $O/prof_$tag.err)
done
run() {
  tag=$1; lib=$2
  THX_LIB=$R/$lib timeout -k 10 300 python -u $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline \
      --no-extras > $O/$tag.json 2> $O/$tag.err
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print(json.dumps({'tag': '$tag', 'value': d['value'], 'ms_per_step': d['ms_per_step']}))" >> $O/ab.jsonl
}
run new thunder_amd/libthunder_amd.so
run old thunder_amd/ab/lib_cdfglob.so
run new_b thunder_amd/libthunder_amd.so
run old_b thunder_amd/ab/lib_cdfglob.so
