#!/bin/bash
# Timing-only decomposition of the warp-specialised conv (ablib/libcwdm_diag.so,
# tools/build_ab_lib.sh diag HEAD V5DIAG=1): conv_bench per CWDM_V5_DIAGMASK.
# usage: tools/gpu_v5diag.sh TAG "CASE:MASK[:ENV=..]" ...
set -o pipefail
T=${1:-v5diag}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
for spec in "$@"; do
  IFS=: read -r case mask extra <<< "$spec"
  r=$(env CWDM_LIB=ablib/libcwdm_diag.so CWDM_ALLOW_STALE_LIB=1 CWDM_V5_DIAGMASK=$mask $extra \
      timeout -k 10 120 python -u tools/conv_bench.py --iters 20 --only $case 2>&1) || { echo "$r" | tail -5; exit 1; }
  echo "mask=$mask $extra :: $r" | tee -a $O/diag.txt
done
