#!/bin/bash
# conv micro-benchmark under rocprofv3 kernel trace.  usage: tools/gpu_convprof.sh TAG [conv_bench args]
set -e -o pipefail
T=${1:-cp}; shift || true
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 200 python -u tools/conv_bench.py "$@" > $O/conv_bench.txt 2>&1
cat $O/conv_bench.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/tools/conv_bench.py "$@" > $O/trace.log 2>&1
find $O/trace -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-160 | head -30
