#!/bin/bash
# one iteration: GPU tests matching a -k filter, then the step's kernel trace
# usage: tools/gpu_iter2.sh TAG "PYTEST_K" [ENV ...]
set -e -o pipefail
T=$1; K=$2; shift 2
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu_trace2.sh ${T}_tr "${@:-CWDM_V5=3}"
