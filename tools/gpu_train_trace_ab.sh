#!/bin/bash
# training parity tests, then per-kernel training-step stats (rocprofv3 kernel trace of
# tools/train_bench.py) for the tree library and ablib/libcwdm_$BASE.so, same box.
# usage: tools/gpu_train_trace_ab.sh TAG BASE
set -e -o pipefail
T=$1; BASE=$2
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_ddp.py > $O/pytest_train.log 2>&1 || { tail -30 $O/pytest_train.log; exit 1; }
tail -1 $O/pytest_train.log
CWDM_LIB=ablib/libcwdm_$BASE.so CWDM_ALLOW_STALE_LIB=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/base -o run --output-format csv -- python3 $R/tools/train_bench.py --steps 3 --warmup 1 > $O/base.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tree -o run --output-format csv -- python3 $R/tools/train_bench.py --steps 3 --warmup 1 > $O/tree.log 2>&1
tail -1 $O/base.log; tail -1 $O/tree.log
