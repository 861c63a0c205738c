set -e -o pipefail
# config 5 A/B: the 28^3 64-channel down-block convs (K-split target) and the
# 56^3 64-channel convs (v5 tiles-per-CU threshold), per conv and per step
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-c5ab}; mkdir -p $O; cd $R
B="--steps 3 --warmup 1 --cpu-baseline 0 --respaced 0 --batched 0 --fp32 0 --fp32x 0 --train 0 --wavunet 0 --train5 0 --fp16 0 --config5 20"
for env in "X=0" "CWDM_V4_KSPLIT_TARGET=64" "CWDM_V5_MIN_TPC=1" "CWDM_V4_KSPLIT_TARGET=64 CWDM_V5_MIN_TPC=1"; do
  echo "== $env"
  env $env timeout -k 10 120 python -u tools/conv_bench.py --only C5_ --iters 20 2>/dev/null | tee -a $O/cb.txt
  env $env timeout -k 10 300 python -u bench.py $B > $O/b.json 2> $O/b.err
  python -c "import json;d=json.load(open('$O/b.json'))['config5_224'];print('config5', d['ms_per_step'], d['mfma_frac'])"
done
