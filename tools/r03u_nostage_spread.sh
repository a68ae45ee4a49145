set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03u; mkdir -p $O
cd $R
for ru in 24 48; do for sp in 0.5 1.5 3 8 0; do for L in "" thunder_amd/ab/lib_nostage.so; do
  lib=${L:-thunder_amd/libthunder_amd.so}
  THX_LIB=$lib timeout -k 10 120 python tools/microbench.py local --ru $ru --spread $sp --images 4096 --reps 5 | sed "s|^{|{\"lib\": \"$(basename $lib)\", \"spread\": $sp, |" >> $O/ab.jsonl || exit 4
done; done; done
echo done
