#!/bin/bash
# training-step kernel trace only (tools/train_bench.py under rocprofv3 --kernel-trace --stats)
# usage: tools/gpu_train_trace.sh TAG [train_bench args]
set -e -o pipefail
T=${1:-tt}; shift || true
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/tools/train_bench.py --steps 2 --warmup 1 "$@" > $O/trace.log 2>&1
tail -1 $O/trace.log
