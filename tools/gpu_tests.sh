#!/bin/bash
# GPU parity tests only (optionally a subset).  usage: tools/gpu_tests.sh TAG [pytest args...]
set -e -o pipefail
T=${1:-t}; shift || true
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 240 --timeout-method thread "${@:-tests}" > $O/pytest.log 2>&1
tail -3 $O/pytest.log
