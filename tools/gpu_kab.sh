#!/bin/bash
# kernel tests + conv_bench (cases matching $2) under env arms, then the bench A/B.
# usage: tools/gpu_kab.sh TAG CASE_FILTER "ENV=a" "ENV=b" ...
set -e -o pipefail
T=$1; F=$2; shift 2
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 240 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_unet.py > $O/pytest.log 2>&1
tail -1 $O/pytest.log
for cfg in "$@"; do
  echo "== $cfg"; env $cfg timeout -k 10 200 python -u tools/conv_bench.py --only "$F" 2>&1 | grep -v amdgpu
done
bash tools/gpu_ab_quick.sh $T "$@"
