# bench-launch PMC (L1/L2 lines) + rocprof kernel stats of the bench, for profiles/
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r03j; mkdir -p $O
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum \
    --kernel-include-regex "k_local_fused" --output-format csv -d $O/pmc_lines -o run \
    -- python3 $R/bench.py --steps 1 --warmup 0 --no-extras --no-cpu-baseline > $O/pmc_lines.log 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
    -- python3 $R/bench.py --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err || exit 3
echo done
