#!/bin/bash
CASE=$1; OUT=$2
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/$OUT
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQC_TC_INST_REQ SQC_TC_STALL SQ_WAVES -d $R/$OUT/p1 -o pmc --output-format csv -- python3 $R/tools/conv_bench.py --iters 3 --only $CASE > $R/$OUT/p1.log 2>&1
