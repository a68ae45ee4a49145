set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03n; mkdir -p $O
cd $R
for L in "" thunder_amd/ab/lib_oldcells.so; do
  THX_LIB=${L:-thunder_amd/libthunder_amd.so} timeout -k 10 500 python tools/config_bench.py --only C5,C5cells,C5n,C5ncells | sed "s|^{|{\"lib\": \"$(basename ${L:-new})\", |" >> $O/configs.jsonl 2>>$O/configs.err || exit 3
  for sp in 0 3 1.5; do
  THX_LIB=${L:-thunder_amd/libthunder_amd.so} timeout -k 10 120 python tools/microbench.py local --box 256 --ru 126 --images 512 --spread $sp --cells 1 --reps 3 | sed "s|^{|{\"lib\": \"$(basename ${L:-new})\", |" >> $O/fullres.jsonl 2>>$O/configs.err || exit 4
  done
done
echo done
