#!/bin/bash
# conv_bench under several env settings.  usage: tools/gpu_ab_conv.sh TAG "ENV1" "ENV2" ... (ENV = "A=1 B=2" or "-")
set -e -o pipefail
T=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
i=0
for e in "$@"; do
  i=$((i+1))
  echo "== $e" | tee -a $O/ab.txt
  if [ "$e" = "-" ]; then e=""; fi
  env $e timeout -k 10 200 python -u tools/conv_bench.py --iters 20 ${CONV_ONLY:+--only $CONV_ONLY} > $O/run$i.txt 2>&1
  cat $O/run$i.txt | tee -a $O/ab.txt
done
