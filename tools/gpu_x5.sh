#!/bin/bash
set -e -o pipefail
T=${1:-x5}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 240 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_sampler_fused.py tests/test_gpu_wavelet2.py tests/test_gpu_unet.py tests/test_gpu_train.py > $O/pytest.log 2>&1
tail -1 $O/pytest.log
timeout -k 10 200 python -u tools/wgrad_bench.py --dma 2>&1 | grep -v amdgpu | tee $O/wg.txt
timeout -k 10 200 python -u tools/conv_bench.py --only L 2>&1 | grep -v amdgpu | grep -E "L3|L4|C5" | tee $O/cb.txt
bash tools/gpu_ab_quick.sh $T "CWDM_SAMPLER2_LDS=1"
