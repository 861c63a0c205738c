#!/bin/bash
# config-5 sampling-step kernel trace: bench.py with only the config5 leg
set -e -o pipefail
T=${1:-c5}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 \
  --cpu-baseline 0 --respaced 0 --batched 0 --train 0 --fp32 0 --fp16 0 --config5 6 --wavunet 0 --train5 0 > $O/bench.log 2>&1
grep -o '"config5_224": {[^}]*' $O/bench.log | head -c 600
