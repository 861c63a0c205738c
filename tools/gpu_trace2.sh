#!/bin/bash
# kernel-trace step timelines: the accurate fast mode (fp32x) step and the training step.
# usage: tools/gpu_trace2.sh TAG
set -e -o pipefail
TAG=${1:-t2}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
SIDE="--cpu-baseline 0 --respaced 0 --batched 0 --train 0 --fp32 0 --fp32x 0 --fp16 0 --config5 0 --wavunet 0 --train5 0"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_x -o run --output-format csv -- python3 $R/bench.py --dtype fp32x --steps 3 --warmup 1 $SIDE > $O/trace_x.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_train -o run --output-format csv -- python3 $R/tools/train_bench.py --steps 3 --warmup 1 > $O/trace_train.log 2>&1
cd $R
python3 tools/trace_step.py $O/trace_x --last > $O/x_step_timeline.txt
python3 tools/trace_step.py $O/trace_train --last > $O/train_timeline.txt
tail -25 $O/x_step_timeline.txt
