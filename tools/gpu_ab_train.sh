#!/bin/bash
# Same-box A/B of env settings on the config-3 training step: tools/train_bench.py (ms per step,
# 5 steps, twice, alternating) and one kernel trace per setting, aggregated by kernel name.
# usage: tools/gpu_ab_train.sh TAG "ENV1=a" "ENV2=b" ...   ("-" = no env change)
set -e -o pipefail
T=$1; shift; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
for rep in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i+1)); e=$cfg; [ "$e" = "-" ] && e=""
    env $e timeout -k 10 300 python -u tools/train_bench.py --steps 5 > $O/t_${i}_$rep.json 2> $O/t_${i}_$rep.err
    python3 -c "import json; d=json.loads(open('$O/t_${i}_$rep.json').read().strip().splitlines()[-1]); print('$cfg', d['ms_per_step'])"
  done
done
cd /tmp && export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i+1)); e=$cfg; [ "$e" = "-" ] && e=""; e=${e//=ablib\//=$R/ablib/}
  env $e timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_$i -o run --output-format csv -- python3 $R/tools/train_bench.py --steps 3 --warmup 1 > $O/tr_$i.log 2>&1
  python3 $R/tools/trace_step.py $O/tr_$i --last > $O/step_$i.txt
  echo "== $cfg"; grep -A24 '^total' $O/step_$i.txt
done
