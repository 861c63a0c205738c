#!/bin/bash
# kernel trace of the config-5 leg (224^3, 2-level wavelets, fp16): last step's timeline
set -e -o pipefail
T=${1:-c5}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O
SIDE="--cpu-baseline 0 --respaced 0 --batched 0 --train 0 --fp32 0 --fp32x 0 --fp16 0 --wavunet 0 --train5 0"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 $SIDE --config5 6 > $O/trace.log 2>&1
python3 $R/tools/trace_step.py $O/trace --last > $O/timeline.txt
tail -40 $O/timeline.txt
