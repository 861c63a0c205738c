#!/bin/bash
# One GPU call: parity suite, bench line, rocprofv3 kernel-trace stats and the
# HBM / MFMA PMC passes (one counter group per run) of the sampling bench, and
# the training step (train_bench line + its kernel-trace stats).
# usage: tools/gpu_round.sh TAG [skip-tests]
set -e -o pipefail
TAG=${1:-r04}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
  tail -3 $O/pytest_gpu.log
fi
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err && timeout -k 10 200 python -u tools/volume_bench.py > $O/volume_bench.json 2>&1
tail -1 $O/bench.json | cut -c1-300
timeout -k 10 300 python -u tools/train_bench.py --steps 5 > $O/train_bench.json 2> $O/train_bench.err
tail -1 $O/train_bench.json
SIDE="--cpu-baseline 0 --respaced 0 --batched 0 --train 0 --fp32 0 --fp32x 0 --fp16 0 --config5 0 --wavunet 0 --train5 0"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 $SIDE > $O/trace.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_train -o run --output-format csv -- python3 $R/tools/train_bench.py --steps 3 --warmup 1 > $O/trace_train.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o pmc --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 $SIDE > $O/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o pmc --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 $SIDE > $O/pmc_write.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_MFMA -d $O/pmc_mfma -o pmc --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 $SIDE > $O/pmc_mfma.log 2>&1
cd $R
python3 tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/pmc_traffic.json
python3 tools/trace_step.py $O/trace --last > $O/step_timeline.txt
python3 tools/trace_step.py $O/trace_train --last > $O/train_timeline.txt
echo done
