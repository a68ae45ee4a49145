#!/bin/bash
# One GPU-box pass: parity tests, headline bench, kernel-trace profile and HBM
# PMC passes of the bench.  Run on the GPU box from the repo root:
#   tools/gpu_round.sh TAG [tests|bench|prof|pmc|lines|probe ...]
#   (default: tests bench prof pmc lines)
# Every step has its own time limit; the first failure ends the script.
set -e
tag=$1; shift
steps=${*:-tests bench prof pmc lines}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
export TMPDIR=/tmp
for s in $steps; do
  case $s in
    tests)
      (cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail 15 --timeout 120 \
          --timeout-method thread > $O/tests.log 2>&1) ;;
    bench)
      (cd $R && timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err) ;;
    prof)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d $O/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline \
          --no-extras > $O/prof.json 2> $O/prof.err)
      # the same command with the secondary kernels (scan / full-res / insert)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d $O/prof_extras -o run -- python3 $R/bench.py --steps 1 --warmup 0 \
          --no-cpu-baseline > $O/prof_extras.json 2> $O/prof_extras.err) ;;
    pmc)
      # HBM bytes: FETCH_SIZE and WRITE_SIZE need separate passes (TCC slots);
      # pass 3 the exact 64 / 128-B request split when the box lists the
      # 128-B counter (rocprofv3 -L), pass 4 the L2 hit rate
      (cd /tmp && timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1) || true
      P3="TCC_HIT_sum TCC_MISS_sum"
      grep -q "TCC_EA0_RDREQ_128B" $O/counters.txt && P3="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum"
      i=0
      for P in "FETCH_SIZE" "WRITE_SIZE" "$P3" "TCC_HIT_sum TCC_MISS_sum"; do
        i=$((i+1))
        [ $i = 4 ] && [ "$P3" = "$P" ] && break
        (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv \
            --kernel-include-regex "k_scan|k_local|k_patch|k_insert|k_prep" \
            -d $O/pmc$i -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline \
            > $O/pmc$i.log 2>&1)
      done
      python3 $R/tools/traffic.py $O $O/traffic.json > /dev/null ;;
    lines)
      # L1 -> L2 line requests of the bench's k_local_fused launches (per phase)
      (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum \
          TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "k_local_fused" --output-format csv \
          -d $O/pmc_lines -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-extras \
          --no-cpu-baseline > $O/pmc_lines.log 2>&1)
      python3 $R/tools/l2_lines.py $O/pmc_lines $O/l2_lines.json > /dev/null ;;
    probe)
      for mb in 0.016 2 16 4096; do
        timeout -k 10 120 $R/tools/probes/l2_roof_bin $mb >> $O/l2_roof.jsonl
      done ;;
  esac
done
