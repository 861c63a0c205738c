#!/bin/bash
# conv_bench A/B over CWDM_V5 modes (0 = v4) on the U-Net conv shapes, then the
# v5 in-kernel stamps (ablib/libcwdm_stamps.so) of a few cases per stamped mode.
# usage: V5LIST="0 2 3" STAMPMODES="2 3" tools/gpu_v5probe.sh TAG [conv_bench --only filter]
set -e -o pipefail
T=$1; F=${2:-L}; V5LIST=${V5LIST:-0 2}; STAMPMODES=${STAMPMODES:-2}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
for v in $V5LIST; do
  CWDM_V5=$v timeout -k 10 300 python -u tools/conv_bench.py --only "$F" 2>/dev/null > $O/cb_$v.txt
  echo "== CWDM_V5=$v"; cat $O/cb_$v.txt
done
if [ -f ablib/libcwdm_stamps.so ]; then
  for m in $STAMPMODES; do
  for c in L0_64_64_gn L0_64_64_nogn L1_128_128_gn; do
    CWDM_V5=$m CWDM_LIB=ablib/libcwdm_stamps.so CWDM_ALLOW_STALE_LIB=1 timeout -k 10 120 python -u tools/v5_stamps.py $c 2>/dev/null > $O/st_${m}_$c.txt
    echo "== stamps CWDM_V5=$m"; cat $O/st_${m}_$c.txt
  done
  done
fi
