#!/bin/bash
# A/B over env settings: config-2 steps/s and config-5 ms/step per setting,
# alternating, twice.  usage: tools/gpu_ab_c25.sh TAG "VAR=a" "VAR=b" ... ("-" = none)
set -e -o pipefail
T=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
OFF="--cpu-baseline 0 --respaced 0 --batched 0 --fp32 0 --fp32x 0 --fp16 0 --train 0 --wavunet 0 --train5 0"
for rep in 1 2; do
  for e in "$@"; do
    [ "$e" = "-" ] && ev="X=0" || ev="$e"
    env $ev timeout -k 10 200 python bench.py --steps 20 --warmup 3 $OFF --config5 0 > $O/c2.json 2> $O/c2.err
    env $ev timeout -k 10 200 python bench.py --steps 1 --warmup 1 $OFF --config5 20 > $O/c5.json 2> $O/c5.err
    echo "$e => c2 $(python -c "import json;d=json.loads(open('$O/c2.json').read().strip().splitlines()[-1]);print(d['value'])") steps/s, c5 $(python -c "import json;d=json.loads(open('$O/c5.json').read().strip().splitlines()[-1]);print(d['config5_224']['ms_per_step'])") ms" | tee -a $O/ab.txt
  done
done
