#!/bin/bash
# r04: default-path kernel trace + full bench line (all side legs)
set -e -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r04b; mkdir -p $O; cd $R
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
tail -1 $O/bench.json
bash tools/gpu_trace2.sh r04b_tr "CWDM_V5=3"
