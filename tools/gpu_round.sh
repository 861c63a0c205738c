#!/bin/bash
# One GPU call: parity suite, bench line, rocprofv3 kernel-trace stats and the
# two HBM PMC passes (FETCH_SIZE / WRITE_SIZE each in its own run) of the bench.
# usage: tools/gpu_round.sh TAG [skip-tests]
set -e -o pipefail
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
  tail -3 $O/pytest_gpu.log
fi
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err && timeout -k 10 200 python -u tools/volume_bench.py > $O/volume_bench.json 2>&1
tail -1 $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --respaced 0 --batched 0 > $O/trace.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o pmc --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-baseline 0 --respaced 0 --batched 0 > $O/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o pmc --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-baseline 0 --respaced 0 --batched 0 > $O/pmc_write.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_MFMA -d $O/pmc_mfma -o pmc --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-baseline 0 --respaced 0 --batched 0 > $O/pmc_mfma.log 2>&1
echo done
