#!/bin/bash
# rocprofv3 kernel trace of a short bench run (sampling leg only) + the per-launch step timeline.
# usage: tools/gpu_trace.sh TAG [ENV...]
set -e -o pipefail
T=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
SIDE="--cpu-baseline 0 --respaced 0 --batched 0 --train 0 --fp32 0 --config5 0 --wavunet 0 --train5 0"
env "$@" X=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 $SIDE > $O/trace.log 2>&1
cd $R && python3 tools/trace_step.py $O/trace > $O/step_timeline.txt && python3 tools/trace_step.py $O/trace --agg > $O/step_agg.txt
cat $O/step_agg.txt | head -30
