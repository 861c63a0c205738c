#!/bin/bash
# The full default bench line (every side figure, CPU baseline) and a
# rocprofv3 kernel trace of the sampling step.  usage: tools/gpu_bench_trace.sh TAG [bench args]
set -e -o pipefail
T=${1:-bt}; shift || true
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python -u bench.py "$@" > $O/bench.json 2> $O/bench.err
tail -1 $O/bench.json | cut -c1-300
SIDE="--cpu-baseline 0 --respaced 0 --batched 0 --train 0 --fp32 0 --fp16 0 --config5 0 --wavunet 0 --train5 0"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 $SIDE > $O/trace.log 2>&1
echo traced
