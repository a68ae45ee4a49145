set -o pipefail
O=gpurun_out/r03h; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -le 1 ] || exit $rc
for k in 0 9; do for br in 0 1; do
  timeout -k 10 120 python tools/microbench.py local --clouds tools/data/clouds_eval.npz --k $k --images 4096 --reps 5 --bricks $br >> $O/ab.jsonl 2>>$O/ab.err || exit 3
done; done
THX_LIB=thunder_amd/ab/lib_count.so timeout -k 10 120 python tools/microbench.py local --clouds tools/data/clouds_eval.npz --k 0 --images 4096 --reps 1 --bricks 1 --counts 1 >> $O/ab.jsonl 2>>$O/ab.err || exit 4
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 5
THX_LIB=thunder_amd/ab/lib_nobricks.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras > $O/bench_nobricks.json 2> $O/bench_nobricks.err || exit 6
echo done
