#!/bin/bash
# Round-3 A/B experiments of the local phase (run on the GPU box from the repo
# root; results under gpurun_out/TAG, copied to profiles/r03_*):
#   tools/r03_experiments.sh TAG STEP...
#   clouds   dump the clouds the bench's phases evaluate (needs
#            thunder_amd/ab_dbg/lib_dumpq.so: tools/build_define.sh dumpq
#            optimiser.hip -DTHX_DUMP_QUAT=1, moved to ab_dbg/)
#   layouts  half-complex vs bricked vs cell projectee on those clouds
#            (tools/data/clouds_eval.npz), phases 0 2 5 9, 4096 images
#   pmc      L1 / L2 / TA counters of the same launches (tools/pmc_gather.sh)
#   fullres  full-resolution phase and C5 in the cell layout, the in-tree
#            library vs thunder_amd/ab/lib_*.so
# The headline measurement set is tools/gpu_round.sh.
set -e
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
cd $R
for s in "$@"; do
  case $s in
    clouds)
      timeout -k 10 240 env THX_LIB=thunder_amd/ab_dbg/lib_dumpq.so python tools/dump_clouds.py 4096 \
          > $O/dump.log 2>&1 ;;
    layouts)
      for k in 0 2 5 9; do
        for lay in "" "--bricks 1" "--cells 1"; do
          timeout -k 10 120 python tools/microbench.py local --clouds tools/data/clouds_eval.npz \
              --k $k --images 4096 --reps 5 $lay >> $O/layouts.jsonl 2>> $O/layouts.err
        done
      done ;;
    pmc)
      timeout -k 10 600 bash tools/pmc_gather.sh gpurun_out/$tag/pmc "0 9" ;;
    fullres)
      for L in "" thunder_amd/ab/*.so; do
        lib=${L:-thunder_amd/libthunder_amd.so}
        THX_LIB=$lib timeout -k 10 500 python tools/config_bench.py --only C5,C5cells,C5n,C5ncells \
            | sed "s|^{|{\"lib\": \"$(basename $lib)\", |" >> $O/configs.jsonl 2>> $O/configs.err
        for sp in 0 3 1.5; do
          THX_LIB=$lib timeout -k 10 120 python tools/microbench.py local --box 256 --ru 126 \
              --images 512 --spread $sp --cells 1 --reps 3 \
              | sed "s|^{|{\"lib\": \"$(basename $lib)\", |" >> $O/fullres.jsonl 2>> $O/configs.err
        done
      done ;;
  esac
done
