#!/bin/bash
# quick GPU check: parity suite, bench line, kernel-trace stats.  usage: tools/gpu_quick.sh TAG
set -e -o pipefail
T=${1:-q}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --cpu-baseline 0 > $O/bench.json 2> $O/bench.err
tail -1 $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 > $O/trace.log 2>&1
echo done
