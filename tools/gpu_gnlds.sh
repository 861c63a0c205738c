#!/bin/bash
# GroupNorm-in-LDS check: DMA-conv + U-Net parity, then bench A/B against the gn_apply pass.
set -e -o pipefail
T=${1:-gnlds}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 240 --timeout-method thread tests/test_gpu_kernels.py -k "dma or fused" > $O/pytest_k.log 2>&1
tail -2 $O/pytest_k.log
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 240 --timeout-method thread tests/test_gpu_unet.py -k "production or wavunet or tiny" > $O/pytest_u.log 2>&1
tail -2 $O/pytest_u.log
CWDM_GN_LDS=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --train 0 --fp32 0 --batched 0 --respaced 0 > $O/bench_off.json 2> $O/bench_off.err
tail -1 $O/bench_off.json | cut -c1-300
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --train 0 --fp32 0 --batched 0 --respaced 0 > $O/bench_on.json 2> $O/bench_on.err
tail -1 $O/bench_on.json | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --respaced 0 --batched 0 --train 0 --fp32 0 > $O/trace.log 2>&1
echo traced
