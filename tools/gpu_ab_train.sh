#!/bin/bash
# A/B of the training step over env settings (alternating, twice): tools/gpu_ab_train.sh "VAR=a" "VAR=b" ...
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/abt; cd $R
for rep in 1 2; do
  for cfg in "$@"; do
    env $cfg timeout -k 10 200 python tools/train_bench.py --steps 5 > gpurun_out/abt/t.json 2>gpurun_out/abt/t.err || exit 1
    echo "$cfg => $(python -c "import json;d=json.loads(open('gpurun_out/abt/t.json').read().strip().splitlines()[-1]);print(d['ms_per_step'])") ms"
  done
done
