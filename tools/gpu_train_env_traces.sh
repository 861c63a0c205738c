#!/bin/bash
# training-step kernel traces under several env settings, same box.
# usage: tools/gpu_train_env_traces.sh TAG "ENV1=a ENV2=b" "ENV1=c" ...  (post-process with train_step_agg.py)
set -e -o pipefail
T=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i+1))
  echo "$i $cfg" >> $O/arms.txt
  env $cfg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$i -o run --output-format csv -- python3 $R/tools/train_bench.py --steps 2 --warmup 1 > $O/trace_$i.log 2>&1
  tail -1 $O/trace_$i.log | cut -c1-200
done
