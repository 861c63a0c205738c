#!/bin/bash
# train_bench under several env settings, same box.  usage: tools/gpu_ab_train.sh TAG "ENV1" "ENV2" ... ("-" = none)
set -e -o pipefail
T=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
i=0
for e in "$@"; do
  i=$((i+1))
  [ "$e" = "-" ] && e=""
  echo "== $e" >> $O/ab.txt
  env $e timeout -k 10 300 python -u tools/train_bench.py --steps 6 > $O/run$i.json 2> $O/run$i.err
  tail -1 $O/run$i.json | cut -c1-200 >> $O/ab.txt
done
cat $O/ab.txt
