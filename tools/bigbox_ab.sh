#!/bin/bash
# big-box A/B: C5 parity tests, C5 throughput (default = big boxes at C5, bignone),
# full-res box-256 local phase (default = normal boxes, bigall)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/bigab
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "c5 or C5 or fullres or full or local_phase" > $O/tests.log 2>&1
timeout -k 10 400 python -u tools/config_bench.py --only C5,C5cells,C5n,C5ncells > $O/c5_default.jsonl 2>> $O/err.log
THX_LIB=$R/thunder_amd/ab/lib_bignone.so timeout -k 10 400 python -u tools/config_bench.py --only C5,C5n > $O/c5_bignone.jsonl 2>> $O/err.log
for L in default lib_bigall.so; do
  if [ "$L" = default ]; then unset THX_LIB; else export THX_LIB=$R/thunder_amd/ab/$L; fi
  for sp in 1.5 3; do
    timeout -k 10 120 python tools/microbench.py local --ru 126 --images 512 --spread $sp --reps 3 | sed "s/}$/, \"lib\": \"$L\"}/" >> $O/fullres256.jsonl 2>> $O/err.log
  done
done
