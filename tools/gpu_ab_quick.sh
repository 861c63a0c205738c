#!/bin/bash
# A/B of env settings on the bench's steps/s.  usage: tools/gpu_ab_quick.sh TAG "ENV1=a ENV2=b" "ENV1=c" ...
set -e -o pipefail
T=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
i=0
for rep in 1 2; do
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 python -u bench.py --cpu-baseline 0 --train 0 --fp32 0 --batched 0 --respaced 0 --steps 30 > $O/ab_$i.json 2> $O/ab_$i.err
  python3 -c "import json,sys; d=json.loads(open('$O/ab_$i.json').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
done
