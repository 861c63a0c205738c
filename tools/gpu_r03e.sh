#!/bin/bash
# round-3 fused head + sampler: new tests, head micro-bench (with / without
# GroupNorm+SiLU), bench sampler line + kernel trace
set -e -o pipefail
T=${1:-r03e}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread \
  tests/test_gpu_sampler_fused.py "tests/test_gpu_unet.py::test_hip_graph_loop_equals_eager_loop" > $O/pytest.log 2>&1 \
  || [ $? -eq 1 ]   # test failures (rc 1) still run the timings below; anything else stops
grep -E "PASSED|FAILED|ERROR" $O/pytest.log | cut -c1-150; tail -2 $O/pytest.log
timeout -k 10 120 python -u tools/conv_bench.py --only L0_64_8_out > $O/head.log 2>&1
cat $O/head.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 \
  --cpu-baseline 0 --respaced 0 --batched 0 --train 0 --fp32 0 --fp16 0 --config5 0 --wavunet 0 --train5 0 > $O/bench.log 2>&1
tail -c 600 $O/bench.log
