#!/bin/bash
# r04 iteration: split-mode + v5 tests, conv_bench over CWDM_V5 modes + stamps, bench A/B
set -e -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r04a; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "split_bf16 or accurate or v5 or dma_kernel" --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
V5LIST="0 2 3" STAMPMODES="2 3" bash tools/gpu_v5probe.sh r04a_probe L0_
bash tools/gpu_iter.sh r04a_bench - "CWDM_V5=0" "CWDM_V5=2" "CWDM_V5=3"
