#!/bin/bash
# In-kernel phase stamps of the warp-specialised conv (ablib/libcwdm_stamps.so,
# tools/build_stamps_lib.sh) per conv_bench case and env setting.
# usage: tools/gpu_v5stamps.sh TAG "CASE[:ENV=..]" ...
set -o pipefail
T=${1:-v5stamps}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
for spec in "$@"; do
  IFS=: read -r case extra <<< "$spec"
  r=$(env CWDM_LIB=ablib/libcwdm_stamps.so CWDM_ALLOW_STALE_LIB=1 $extra \
      timeout -k 10 120 python -u tools/v5_stamps.py $case 2>&1) || { echo "$r" | tail -5; exit 1; }
  echo "== $case $extra" | tee -a $O/stamps.txt
  echo "$r" | grep -v amdgpu.ids | tee -a $O/stamps.txt
done
