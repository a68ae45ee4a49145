set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/csab
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_ctfsearch.py tests/test_gpu_local_iface.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "ctf or local_phase or forwards" > $O/tests.log 2>&1
for nd in 0 3 9; do
  timeout -k 10 120 python tools/microbench.py local --images 12500 --spread 3 --nd $nd --reps 3 >> $O/mb_default.jsonl 2>> $O/mb.err
done
for nd in 3 9; do
  THX_LIB=$R/thunder_amd/ab/lib_cs_nct1.so timeout -k 10 120 python tools/microbench.py local --images 12500 --spread 3 --nd $nd --reps 3 >> $O/mb_nct1.jsonl 2>> $O/mb.err
done
