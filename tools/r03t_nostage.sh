set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03t; mkdir -p $O
cd $R
THX_LIB=thunder_amd/ab/lib_nostage.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -k "(local or phase) and not staged_patches" -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
for k in 0 2 5 9; do for L in "" thunder_amd/ab/lib_nostage.so; do
  lib=${L:-thunder_amd/libthunder_amd.so}
  THX_LIB=$lib timeout -k 10 120 python tools/microbench.py local --clouds tools/data/clouds_eval.npz --k $k --images 4096 --reps 5 | sed "s|^{|{\"lib\": \"$(basename $lib)\", |" >> $O/ab.jsonl || exit 4
done; done
for L in "" thunder_amd/ab/lib_nostage.so; do
  lib=${L:-thunder_amd/libthunder_amd.so}
  THX_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras | sed "s|^{|{\"lib\": \"$(basename $lib)\", |" >> $O/bench.jsonl 2>>$O/bench.err || exit 5
done
echo done
