#!/bin/bash
# Same-box A/B of env settings: the bench line (ms per step, 30 steps, twice, alternating) and one
# kernel trace per setting, aggregated by kernel name (tools/trace_step.py --last).
# usage: tools/gpu_ab_trace.sh TAG "ENV1=a" "ENV2=b" ...   ("-" = no env change)
set -e -o pipefail
T=$1; shift; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
SIDE="--cpu-baseline 0 --respaced 0 --batched 0 --train 0 --fp32 0 --fp32x 0 --fp16 0 --config5 0 --wavunet 0 --train5 0"
for rep in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i+1)); e=$cfg; [ "$e" = "-" ] && e=""
    env $e timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 $SIDE > $O/b_${i}_$rep.json 2> $O/b_${i}_$rep.err
    python3 -c "import json; d=json.loads(open('$O/b_${i}_$rep.json').read().strip().splitlines()[-1]); print('$cfg', d['ms_per_step'])"
  done
done
cd /tmp && export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i+1)); e=$cfg; [ "$e" = "-" ] && e=""; e=${e//=ablib\//=$R/ablib/}
  env $e timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_$i -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $SIDE > $O/tr_$i.log 2>&1
  python3 $R/tools/trace_step.py $O/tr_$i --last > $O/step_$i.txt
  echo "== $cfg"; grep -A14 '^total' $O/step_$i.txt
done
