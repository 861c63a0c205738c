#!/bin/bash
# accurate fast mode (fp32x): its parity tests, the kernel-trace step timeline (rocprofv3, last
# step) and a plain 20-step bench line.  usage: tools/gpu_x_bench.sh TAG
set -e -o pipefail
TAG=${1:-xb}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
SIDE="--cpu-baseline 0 --respaced 0 --batched 0 --train 0 --fp32 0 --fp32x 0 --fp16 0 --config5 0 --wavunet 0 --train5 0"
bash tools/gpu_tests.sh $TAG -k "accurate or fp32x" tests/test_gpu_fullsize.py tests/test_gpu_unet.py
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_x -o run --output-format csv -- python3 $R/bench.py --dtype fp32x --steps 3 --warmup 1 $SIDE > $O/trace_x.log 2>&1)
python3 tools/trace_step.py $O/trace_x --last > $O/x_step_timeline.txt
tail -22 $O/x_step_timeline.txt
timeout -k 10 300 python3 bench.py --dtype fp32x --steps 20 --warmup 3 $SIDE > $O/xbench.log 2>&1
grep -o '"ms_per_step": [0-9.]*' $O/xbench.log
