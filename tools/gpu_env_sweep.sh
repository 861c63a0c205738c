#!/bin/bash
# bench steps/s for several env settings on the same box (2 reps each, interleaved).
# usage: tools/gpu_env_sweep.sh TAG "ENV_1" "ENV_2" ...   ("-" = no env)
set -e -o pipefail
T=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
for rep in 1 2; do
  for e in "$@"; do
    ee=$e; [ "$e" = "-" ] && ee=""
    env $ee timeout -k 10 200 python -u bench.py --cpu-baseline 0 --train 0 --fp32 0 --batched 0 --respaced 0 --config5 0 --wavunet 0 --train5 0 --steps 30 > $O/b.json 2> $O/b.err
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$e', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
