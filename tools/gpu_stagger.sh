for st in 0 -1 20000 40000; do
  echo "stagger=$st" >> gpurun_out/stag.txt
  CWDM_CONV_STAGGER=$st timeout -k 10 60 python tools/conv_bench.py --iters 20 --only L0_64_64_gn >> gpurun_out/stag.txt 2>&1 || exit 1
  CWDM_CONV_STAGGER=$st timeout -k 10 60 python tools/conv_bench.py --iters 20 --only 128_128 >> gpurun_out/stag.txt 2>&1 || exit 1
done
