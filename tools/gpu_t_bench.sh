#!/bin/bash
# GPU tests (subset) then a short bench line and kernel-trace stats.  usage: tools/gpu_t_bench.sh TAG [pytest paths...]
set -e -o pipefail
T=${1:-tb}; shift || true
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 240 --timeout-method thread "${@:-tests}" > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --train 0 --fp32 0 --batched 0 > $O/bench.json 2> $O/bench.err
tail -1 $O/bench.json | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --respaced 0 --batched 0 --train 0 --fp32 0 > $O/trace.log 2>&1
echo traced
