set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03r; mkdir -p $O
cd $R
for cfg in "" "--chunk 6250 --streams 2" "--chunk 4167 --streams 3" "--chunk 3125 --streams 4" "--chunk 6250"; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras $cfg 2>>$O/err.log | sed "s|^{|{\"cfg\": \"$cfg\", |" >> $O/bench.jsonl || exit 3
done
echo done
