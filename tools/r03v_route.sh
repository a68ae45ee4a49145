set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03v; mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log
[ $rc -le 1 ] || exit $rc
for L in "" thunder_amd/ab/lib_pct25.so thunder_amd/ab/lib_pct80.so thunder_amd/ab/lib_noroute.so; do
  lib=${L:-thunder_amd/libthunder_amd.so}
  for sp in 0.5 1.5 3 8 0; do
    THX_LIB=$lib timeout -k 10 120 python tools/microbench.py local --spread $sp --images 4096 --reps 5 | sed "s|^{|{\"lib\": \"$(basename $lib)\", \"spread\": $sp, |" >> $O/ab.jsonl || exit 4
  done
  for k in 0 5 9; do
    THX_LIB=$lib timeout -k 10 120 python tools/microbench.py local --clouds tools/data/clouds_eval.npz --k $k --images 4096 --reps 5 | sed "s|^{|{\"lib\": \"$(basename $lib)\", |" >> $O/ab.jsonl || exit 5
  done
done
for L in "" thunder_amd/ab/lib_noroute.so; do
  lib=${L:-thunder_amd/libthunder_amd.so}
  THX_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras | sed "s|^{|{\"lib\": \"$(basename $lib)\", |" >> $O/bench.jsonl 2>>$O/bench.err || exit 6
done
echo done
