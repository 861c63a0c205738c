#!/bin/bash
# training iteration: train tests (optional -k filter), train_bench line, and the
# training step's kernel trace (per-kernel aggregate of the last step)
# usage: tools/gpu_train.sh TAG [pytest -k filter | -]
set -e -o pipefail
T=${1:-train}; K=${2:-}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
if [ "$K" != "-" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q --timeout 240 --timeout-method thread ${K:+-k "$K"} > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
timeout -k 10 300 python -u tools/train_bench.py --steps 5 > $O/train_bench.json 2> $O/train_bench.err
tail -1 $O/train_bench.json | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_train -o run --output-format csv -- python3 $R/tools/train_bench.py --steps 3 --warmup 1 > $O/trace_train.log 2>&1
python3 $R/tools/trace_step.py $O/trace_train --last > $O/train_timeline.txt
tail -45 $O/train_timeline.txt
