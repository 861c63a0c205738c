#!/bin/bash
# Same-lease A/B of two whole trees (bench.py + library + Python), alternating A, B, A, B,
# then one kernel trace of each step.  Tree A lives under abtree/NAME (tools/build_ab_tree.sh),
# tree B is this one.  usage: tools/gpu_ab_tree.sh TAG NAME [STEPS] [REPS]
set -e -o pipefail
TAG=$1; NAME=$2; STEPS=${3:-50}; REPS=${4:-2}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
A=$R/abtree/$NAME
SIDE="--cpu-baseline 0 --respaced 0 --batched 0 --train 0 --fp32 0 --fp32x 0 --fp16 0 --config5 0 --wavunet 0 --train5 0"
run() {  # tree label rep
  cd $1
  timeout -k 10 240 python -u bench.py --steps $STEPS --warmup 5 $SIDE > $O/$2_$3.json 2> $O/$2_$3.err
  python3 -c "import json; d=json.loads(open('$O/$2_$3.json').read().strip().splitlines()[-1]); print('$2', $3, d['ms_per_step'], d['roofline']['frac'])"
}
for rep in $(seq 1 $REPS); do
  run $A $NAME $rep
  run $R head $rep
done
cd /tmp && export TMPDIR=/tmp
cd $A && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$NAME -o run --output-format csv -- python3 $A/bench.py --steps 5 --warmup 2 $SIDE > $O/trace_$NAME.log 2>&1
cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_head -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 $SIDE > $O/trace_head.log 2>&1
cd $R
python3 tools/trace_step.py $O/trace_$NAME --last > $O/step_timeline_$NAME.txt
python3 tools/trace_step.py $O/trace_head --last > $O/step_timeline_head.txt
echo done
