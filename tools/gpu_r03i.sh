set -o pipefail
O=gpurun_out/r03i; mkdir -p $O
for mb in 2 16; do timeout -k 10 60 tools/probes/l2_roof_bin $mb >> $O/l2_roof.jsonl || exit 2; done
for k in 0 5 9; do for L in "" thunder_amd/ab/lib_pair.so; do for br in 0 1; do
  [ -z "$L" ] || [ $br = 1 ] || continue
  THX_LIB=${L:-thunder_amd/libthunder_amd.so} timeout -k 10 120 python tools/microbench.py local --clouds tools/data/clouds_eval.npz --k $k --images 4096 --reps 5 --bricks $br | sed "s|^{|{\"lib\": \"$(basename ${L:-new})\", |" >> $O/ab.jsonl 2>>$O/ab.err || exit 3
done; done; done
timeout -k 10 600 bash tools/pmc_gather.sh gpurun_out/r03i/pmc "0 9" || exit 4
echo done
