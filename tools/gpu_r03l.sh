set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03l; mkdir -p $O
cd $R
for mb in 0.016 2 16; do timeout -k 10 60 tools/probes/l2_roof_bin $mb >> $O/l2_roof.jsonl || exit 2; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_reconstruct.py tests/test_gpu_insert.py -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1 || exit 3
tail -2 $O/tests.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 4
echo done
