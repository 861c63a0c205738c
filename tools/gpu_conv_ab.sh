#!/bin/bash
# conv parity tests (default kernels), then conv_bench and bench steps/s A/B
# between two env settings.  usage: tools/gpu_conv_ab.sh TAG "ENV_A" "ENV_B"
set -e -o pipefail
T=$1; A=$2; B=$3
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "conv3d or head" > $O/pytest_conv.log 2>&1 || { tail -30 $O/pytest_conv.log; exit 1; }
tail -2 $O/pytest_conv.log
for e in "$A" "$B"; do
  echo "== conv_bench $e"
  env $e timeout -k 10 200 python -u tools/conv_bench.py --iters 20 2>&1 | tee -a $O/conv_bench.txt
done
for rep in 1 2; do
  for e in "$A" "$B"; do
    env $e timeout -k 10 200 python -u bench.py --cpu-baseline 0 --train 0 --fp32 0 --batched 0 --respaced 0 --config5 0 --wavunet 0 --train5 0 --steps 30 > $O/b.json 2> $O/b.err
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$e', d['value'], d['ms_per_step'], d['roofline'])"
  done
done
