#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over one wgrad_bench --dma case.
# usage: tools/pmc_wgrad.sh CASE_INDEX OUTDIR
set -e
C=$1; OUT=$2
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/$OUT
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $R/$OUT/p$i -o pmc --output-format csv -- python3 $R/tools/wgrad_bench.py --dma --case $C > $R/$OUT/p$i.log 2>&1
done
