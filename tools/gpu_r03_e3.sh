#!/bin/bash
# single-round wgrad split: training tests, wgrad micro-bench, training bench
set -e -o pipefail
T=${1:-r03e3}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests/test_gpu_train.py > $O/pytest.log 2>&1 || [ $? -eq 1 ]
grep -cE "PASSED" $O/pytest.log || true; grep -E "FAILED|ERROR" $O/pytest.log | head -20 || true; tail -1 $O/pytest.log
timeout -k 10 200 python -u tools/wgrad_bench.py --dma > $O/wgrad.log 2>&1; cat $O/wgrad.log
timeout -k 10 300 python -u tools/train_bench.py --steps 5 --warmup 2 > $O/train.log 2>&1; tail -1 $O/train.log | head -c 300
