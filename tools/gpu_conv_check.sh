set -o pipefail
timeout -k 10 240 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "dma or gn_apply or fused" > gpurun_out/t_v4.log 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/t_v4.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python tools/conv_bench.py --iters 20 > gpurun_out/cb_v4.txt 2>&1 && CWDM_CONV_PATH=1 timeout -k 10 120 python tools/conv_bench.py --iters 20 > gpurun_out/cb_legacy.txt 2>&1
