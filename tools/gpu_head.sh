set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_unet.py -x -q --timeout 120 --timeout-method thread -k "head or dma or production or fused" > gpurun_out/t_head.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_head.log; exit 1; }
tail -2 gpurun_out/t_head.log
timeout -k 10 240 python bench.py --steps 20 --warmup 3 > gpurun_out/b_head.log 2>&1 && tail -1 gpurun_out/b_head.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_head -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 8 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/p_head.log 2>&1
