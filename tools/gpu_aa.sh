#!/bin/bash
# apply-ahead bring-up: its bit-exact tests, conv_bench cases with it off / on / on at helper
# priority 1, and the bench line with it off / on.  usage: tools/gpu_aa.sh TAG [full]
set -e -o pipefail
T=${1:-aa}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k apply_ahead > $O/pytest_aa.log 2>&1
tail -2 $O/pytest_aa.log
if [ "$2" = "full" ]; then
  timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_unet.py tests/test_gpu_fullsize.py -k "v5 or dma or production_unet_forward or fullsize" > $O/pytest_v5.log 2>&1
  tail -2 $O/pytest_v5.log
fi
for c in L0_128_128_gn L0_192_64_cat L1_256_128_cat L0_64_64_gn; do
  for e in "CWDM_V5_AA=0" "CWDM_V5_AA=1" "CWDM_V5_AA=1 CWDM_V5_AA_PRIO=1"; do
    r=$(env $e timeout -k 10 120 python -u tools/conv_bench.py --iters 20 --only $c 2>&1 | grep -v amdgpu)
    echo "$e :: $r" | tee -a $O/conv_ab.txt
  done
done
for e in "CWDM_V5_AA=0" "CWDM_V5_AA=1" "CWDM_V5_AA=1 CWDM_V5_AA_PRIO=1"; do
  env $e timeout -k 10 300 python -u bench.py --cpu-baseline 0 --respaced 0 --batched 0 --train 0 --fp32 0 --fp32x 0 --fp16 0 --config5 0 --wavunet 0 --train5 0 > $O/bench.json 2>&1
  echo "$e :: $(tail -1 $O/bench.json | cut -c100-190)" | tee -a $O/bench_ab.txt
done
