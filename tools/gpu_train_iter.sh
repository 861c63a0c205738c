#!/bin/bash
# training iteration: training GPU tests, then the step's kernel trace
# usage: tools/gpu_train_iter.sh TAG [pytest -k expr]
set -e -o pipefail
T=${1:-ti}; K=${2:-}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 240 --timeout-method thread tests/test_gpu_train.py -k "$K" > $O/pytest.log 2>&1
else
  timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 240 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_ddp.py > $O/pytest.log 2>&1
fi
tail -2 $O/pytest.log
bash tools/gpu_train_trace.sh $T
