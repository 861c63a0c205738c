#!/bin/bash
# config-5 kernel traces: the sampling step (bench.py config5 leg only) and the
# training step (train5 leg only).  usage: tools/gpu_c5_iter.sh TAG
set -e -o pipefail
T=${1:-c5}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
OFF="--cpu-baseline 0 --respaced 0 --batched 0 --train 0 --fp32 0 --fp16 0 --wavunet 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 \
  $OFF --config5 6 --train5 0 > $O/bench.log 2>&1
grep -o '"config5_224": {[^}]*' $O/bench.log | head -c 400; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace5 -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 \
  $OFF --config5 0 --train5 2 > $O/bench5.log 2>&1
grep -o '"train_config5_224": {[^}]*' $O/bench5.log | head -c 400; echo
