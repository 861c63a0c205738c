#!/bin/bash
# small-grid conv time decomposition (timing-only build: tools/build_ab_lib.sh sgdiag HEAD SGDIAG=1):
# conv_bench per CWDM_SG_DIAGMASK (1 no MFMAs, 2 no halo DMA, 4 no weight DMA, 8 no operand reads),
# then the bench step's kernel trace per mask (the in-step, cold-cache times).  usage: tools/gpu_sgdiag.sh TAG MASK...
set -e -o pipefail
T=$1; shift; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
export CWDM_LIB=$R/ablib/libcwdm_sgdiag.so CWDM_ALLOW_STALE_LIB=1
for m in "$@"; do
  for c in L3_256_256_gn L4_256_256_gn L4_256_256_nogn; do
    r=$(CWDM_SG_DIAGMASK=$m timeout -k 10 120 python -u tools/conv_bench.py --iters 50 --only $c 2>&1 | grep -v amdgpu | head -1)
    echo "mask $m :: $r" | tee -a $O/sg_diag.txt
  done
done
SIDE="--cpu-baseline 0 --respaced 0 --batched 0 --train 0 --fp32 0 --fp32x 0 --fp16 0 --config5 0 --wavunet 0 --train5 0"
cd /tmp && export TMPDIR=/tmp
for m in "$@"; do
  CWDM_SG_DIAGMASK=$m timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_$m -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $SIDE > $O/trace_$m.log 2>&1
  python3 $R/tools/trace_step.py $O/trace_$m --last > $O/step_$m.txt
  echo "mask $m: $(grep -E 'conv3d_sg_kernel|gn_fin_apply' $O/step_$m.txt | grep -E '^ +[0-9.]+ us' | tr -s ' ' | tr '\n' ';')"
done
