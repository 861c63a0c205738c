#!/bin/bash
# One GPU call for a kernel iteration: a pytest selection, then bench.py A/B over
# env settings (two reps each).  usage: tools/gpu_iter.sh TAG "PYTEST_K" "ENV1=a" "ENV2=b" ...
# (PYTEST_K "-" skips the tests; no env args skips the bench)
set -e -o pipefail
T=$1; K=$2; shift; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
if [ "$K" != "-" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
i=0
for rep in 1 2; do
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 240 python -u bench.py --cpu-baseline 0 --train 0 --fp32 0 --fp32x 0 --batched 0 --respaced 0 --fp16 0 --config5 0 --wavunet 0 --train5 0 --steps 30 > $O/ab_$i.json 2> $O/ab_$i.err || { tail -20 $O/ab_$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/ab_$i.json').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
done
