#!/bin/bash
# in-kernel phase stamps of the DMA conv for several conv_bench cases (needs ablib/libcwdm_stamps.so,
# built with make STAMPS=1).  usage: tools/gpu_stamps.sh TAG CASE...
set -e -o pipefail
T=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
for c in "$@"; do
  CWDM_LIB=ablib/libcwdm_stamps.so CWDM_ALLOW_STALE_LIB=1 timeout -k 10 120 python -u tools/conv_stamps.py $c 2>&1 | grep -v amdgpu.ids | tee -a $O/stamps.txt
done
