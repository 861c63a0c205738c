set -e -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r04_v5exp; mkdir -p $O; cd $R
for c in L0_64_64_nogn L1_64_64_nogn L0_128_64_nogn L1_128_128_nogn; do
  CWDM_LIB=ablib/libcwdm_stamps.so CWDM_ALLOW_STALE_LIB=1 timeout -k 10 120 python -u tools/v5_stamps.py $c 2>/dev/null > $O/st_$c.txt
  head -12 $O/st_$c.txt
done
