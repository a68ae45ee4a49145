# round-3 measurement set: GPU tests, bench, PMC line traffic and rocprof stats of the bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03k; mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -le 1 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum \
    --kernel-include-regex "k_local_fused" --output-format csv -d $O/pmc_lines -o run \
    -- python3 $R/bench.py --steps 1 --warmup 0 --no-extras --no-cpu-baseline > $O/pmc_lines.log 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
    -- python3 $R/bench.py --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err || exit 3
cd $R && timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 4
echo done
