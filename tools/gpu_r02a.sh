#!/bin/bash
# round-2 check: new training/DDP parity tests, the full bench line, the 2-rank rehearsal
set -e -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r02a; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -m gpu -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_ddp.py > $O/pytest.log 2>&1
tail -3 $O/pytest.log
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err
tail -1 $O/bench.json
CWDM_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 --cpu-baseline 0 --batched 0 --fp32 0 > $O/bench_rehearse2.json 2> $O/bench_rehearse2.err
tail -1 $O/bench_rehearse2.json
