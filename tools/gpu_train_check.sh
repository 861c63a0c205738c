#!/bin/bash
# training-path parity tests then the train_bench line and its kernel-trace stats.  usage: tools/gpu_train_check.sh TAG
set -e -o pipefail
T=${1:-tc}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_ddp.py tests/test_gpu_unet.py > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/train_bench.py --steps 5 > $O/train_bench.json 2> $O/train_bench.err
tail -1 $O/train_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_train -o run --output-format csv -- python3 $R/tools/train_bench.py --steps 3 --warmup 1 > $O/trace_train.log 2>&1
echo traced
