#!/bin/bash
# training parity tests on the tree's library, then train_bench, same box, tree
# library vs ablib/libcwdm_$BASE.so.  usage: tools/gpu_train_ab.sh TAG BASE
set -e -o pipefail
T=$1; BASE=$2
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_ddp.py > $O/pytest_train.log 2>&1 || { tail -30 $O/pytest_train.log; exit 1; }
tail -1 $O/pytest_train.log
A="CWDM_LIB=ablib/libcwdm_$BASE.so CWDM_ALLOW_STALE_LIB=1"
for rep in 1 2; do
  for e in "$A" "-"; do
    ee=$e; [ "$e" = "-" ] && ee=""
    env $ee timeout -k 10 300 python -u tools/train_bench.py --steps 5 > $O/t.json 2> $O/t.err
    python3 -c "import json; d=json.loads(open('$O/t.json').read().strip().splitlines()[-1]); print('${e:0:30}', d['value'], d['ms_per_step'])"
  done
done
