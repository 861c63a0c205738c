#!/bin/bash
# kernels + config 5 + training tests, then the config-5 trace and the training bench / trace
set -e -o pipefail
T=${1:-r03c}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_wavelet2.py tests/test_gpu_train.py > $O/pytest.log 2>&1 || [ $? -eq 1 ]
grep -cE "PASSED" $O/pytest.log || true; grep -E "FAILED|ERROR" $O/pytest.log | head -20 || true; tail -2 $O/pytest.log
bash tools/gpu_c5_trace.sh $T
timeout -k 10 300 python -u tools/train_bench.py --steps 5 --warmup 2 > $O/train.log 2>&1
tail -1 $O/train.log | head -c 300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ttrace -o run --output-format csv -- python3 $R/tools/train_bench.py --steps 3 --warmup 1 > $O/ttrace.log 2>&1
