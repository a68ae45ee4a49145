# A/B of two library builds on the bench: tools/_ab_bench.sh TAG LIB_A LIB_B
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for v in A B; do
    L=$2; [ $v = B ] && L=$3
    THX_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err
  done
done
