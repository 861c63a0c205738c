#!/bin/bash
# conv parity tests on the tree's library, then conv_bench + bench steps/s, same box,
# tree library vs ablib/libcwdm_$BASE.so.  usage: tools/gpu_lib_ab.sh TAG BASE [pytest -k expr]
set -e -o pipefail
T=$1; BASE=$2; K=${3:-"conv3d or head"}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "$K" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
A="CWDM_LIB=ablib/libcwdm_$BASE.so CWDM_ALLOW_STALE_LIB=1"
for e in "$A" "-"; do
  echo "== conv_bench $e"
  [ "$e" = "-" ] && e=""
  env $e timeout -k 10 200 python -u tools/conv_bench.py --iters 20 2>&1 | grep -v amdgpu.ids | tee -a $O/conv_bench.txt
done
for rep in 1 2; do
  for e in "$A" "-"; do
    ee=$e; [ "$e" = "-" ] && ee=""
    env $ee timeout -k 10 200 python -u bench.py --cpu-baseline 0 --train 0 --fp32 0 --batched 0 --respaced 0 --config5 0 --wavunet 0 --train5 0 --steps 30 > $O/b.json 2> $O/b.err
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('${e:0:30}', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
