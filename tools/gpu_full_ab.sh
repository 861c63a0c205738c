#!/bin/bash
# full -m gpu suite, then bench steps/s A/B of two env settings on the same box and a kernel trace.
# usage: tools/gpu_full_ab.sh TAG "ENV_A" "ENV_B"
set -e -o pipefail
T=$1; A=$2; B=$3
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 240 --timeout-method thread tests > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for e in "$A" "$B"; do
    ee=$e; [ "$e" = "-" ] && ee=""
    env $ee timeout -k 10 200 python -u bench.py --cpu-baseline 0 --train 0 --fp32 0 --batched 0 --respaced 0 --config5 0 --wavunet 0 --train5 0 --steps 30 > $O/b.json 2> $O/b.err
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$e', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
bash tools/gpu_trace.sh $T/tr
