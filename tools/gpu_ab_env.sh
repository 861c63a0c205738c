#!/bin/bash
# A/B over env settings of bench.py (alternating, twice): tools/gpu_ab_env.sh "VAR=a VAR2=b" "VAR=c" ...
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/ab; cd $R
for rep in 1 2; do
  for cfg in "$@"; do
    env $cfg timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 --respaced 0 --batched 0 --fp32 0 --fp16 0 --train 0 --config5 0 --wavunet 0 --train5 0 > gpurun_out/ab/ab.json 2>gpurun_out/ab/ab.err || exit 1
    echo "$cfg => $(python -c "import json;d=json.loads(open('gpurun_out/ab/ab.json').read().strip().splitlines()[-1]);print(d['value'])")"
  done
done
