#!/bin/bash
# Kernel traces of the sampling step under several env settings (one rocprofv3
# run each).  usage: tools/gpu_trace2.sh TAG "ENV1=a" "ENV2=b" ...
set -e -o pipefail
T=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O
SIDE="--cpu-baseline 0 --respaced 0 --batched 0 --train 0 --fp32 0 --fp32x 0 --fp16 0 --config5 0 --wavunet 0 --train5 0"
cd /tmp && export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$i -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 $SIDE > $O/trace_$i.log 2>&1
  python3 $R/tools/trace_step.py $O/trace_$i --last > $O/timeline_$i.txt
  echo "== $cfg"; tail -25 $O/timeline_$i.txt
done
