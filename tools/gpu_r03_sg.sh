#!/bin/bash
# partial-brick small-grid kernel: conv kernel tests, config-5 tests, then the config-5 trace
set -e -o pipefail
T=${1:-r03s}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_wavelet2.py > $O/pytest.log 2>&1 || [ $? -eq 1 ]
grep -cE "PASSED" $O/pytest.log || true; grep -E "FAILED|ERROR" $O/pytest.log | head -20 || true; tail -2 $O/pytest.log
bash tools/gpu_c5_trace.sh $T
