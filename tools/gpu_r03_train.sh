#!/bin/bash
# round 3 training: wgrad (incl. the kept-activation DMA path) and U-Net
# backward tests, then the per-kernel training-step trace (tools/train_bench.py)
set -e -o pipefail
T=${1:-r03t}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread \
  tests/test_gpu_train.py > $O/pytest.log 2>&1 || [ $? -eq 1 ]
grep -cE "PASSED" $O/pytest.log || true; grep -E "FAILED|ERROR" $O/pytest.log | head -20 || true; tail -2 $O/pytest.log
grep -E "kept vs recompute|worst grads" $O/pytest.log | head || true
timeout -k 10 300 python -u tools/train_bench.py --steps 5 --warmup 2 > $O/train.log 2>&1
tail -2 $O/train.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/tools/train_bench.py --steps 3 --warmup 1 > $O/trace.log 2>&1
tail -1 $O/trace.log
