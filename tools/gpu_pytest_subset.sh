#!/bin/bash
# A subset of the GPU tests with their printed output kept (-s):
# usage: tools/gpu_pytest_subset.sh TAG "<pytest -k expression or node ids>" [more pytest args]
set -e -o pipefail
T=${1:-t}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest -m gpu -x -v -s --timeout 400 --timeout-method thread "$@" > $O/pytest.log 2>&1
tail -3 $O/pytest.log
