#!/bin/bash
# head conv iteration: sampler / head tests, a kernel trace of the sampling step
# and a FETCH_SIZE pass.  usage: tools/gpu_head_iter.sh TAG
set -e -o pipefail
T=${1:-hd}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 240 --timeout-method thread tests/test_gpu_sampler_fused.py tests/test_gpu_kernels.py -k "head or sampler or fused" > $O/pytest.log 2>&1
tail -1 $O/pytest.log
SIDE="--cpu-baseline 0 --respaced 0 --batched 0 --train 0 --fp32 0 --fp16 0 --config5 0 --wavunet 0 --train5 0"
timeout -k 10 300 python -u bench.py --steps 20 $SIDE > $O/bench.json 2> $O/bench.err
tail -1 $O/bench.json | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 $SIDE > $O/trace.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o pmc --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 $SIDE > $O/pmc_fetch.log 2>&1
echo done
