#!/bin/bash
# wgrad_bench under several env settings, same box.  usage: [WB_ARGS=--dma] tools/gpu_ab_wgrad.sh TAG "ENV1" ... ("-" = none)
set -e -o pipefail
T=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
for e in "$@"; do
  echo "== $e" >> $O/ab.txt
  [ "$e" = "-" ] && e=""
  env $e timeout -k 10 200 python -u tools/wgrad_bench.py ${WB_ARGS:-} 2>&1 | grep wgrad >> $O/ab.txt
done
cat $O/ab.txt
