#!/bin/bash
# v5 drain change: v5 / dma tests, conv_bench residual cases, step trace
set -e -o pipefail
T=${1:-v5res}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "v5 or dma_kernel or production or fullsize_denoising or split_bf16" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/conv_bench.py --only L0_64_64 2>/dev/null > $O/cb.txt; cat $O/cb.txt
bash tools/gpu_trace2.sh ${T}_tr "CWDM_V5=3"
