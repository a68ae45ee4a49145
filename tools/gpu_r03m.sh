set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03m; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ctfsearch.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -le 1 ] || exit $rc
for k in 0 2 5 9; do for cells in 0 1; do
  timeout -k 10 120 python tools/microbench.py local --clouds tools/data/clouds_eval.npz --k $k --images 4096 --reps 5 --cells $cells >> $O/ab.jsonl 2>>$O/ab.err || exit 3
done; done
echo done
