set -e
O=gpurun_out/r05d; mkdir -p $O
for t in prod x6v1 x6v2 x6v3; do
  lib=thunder_amd/ab/lib_$t.so; [ $t = prod ] && lib=thunder_amd/libthunder_amd.so
  THX_LIB=$lib timeout -k 10 120 python -u tools/scan_diff.py > $O/diff_$t.jsonl 2>> $O/err.log
  for k in 1 2; do THX_LIB=$lib timeout -k 10 120 python -u tools/microbench.py scan --algo 4 2>>$O/err.log | tail -1 | sed "s/^/{\"tag\":\"$t\",\"run\":/; s/$/}/" >> $O/time.jsonl; done
done
