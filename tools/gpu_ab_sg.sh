#!/bin/bash
# small-grid conv A/B: conv_bench's 16^3 / 8^3 / config-5 14^3 cases and the bench line per env.
# usage: tools/gpu_ab_sg.sh TAG "ENV1" "ENV2" ...
set -e -o pipefail
T=$1; shift; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
for e in "$@"; do
  for c in L3_256_256_gn L3_256_256_res L4_256_256_gn L4_256_256_nogn C5_L2_128_128_gn; do
    r=$(env $e timeout -k 10 120 python -u tools/conv_bench.py --iters 50 --only $c 2>&1 | grep -v amdgpu | head -1)
    echo "$e :: $r" | tee -a $O/sg_ab.txt
  done
done
for rep in 1 2; do
for e in "$@"; do
  env $e timeout -k 10 300 python -u bench.py --cpu-baseline 0 --respaced 0 --batched 0 --train 0 --fp32 0 --fp32x 0 --fp16 0 --wavunet 0 --train5 0 > $O/bench.json 2>&1
  echo "$e :: $(tail -1 $O/bench.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config5_224"]["ms_per_step"])')" | tee -a $O/bench_ab.txt
done
done
