set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/dbg5
CWDM_V5=2 CWDM_V5_ONLY=0 CWDM_V5_SYNC=1 timeout -k 10 120 python -u tools/dbg_trace.py where 16 16 32 > gpurun_out/dbg5/where_sync.txt 2>&1; echo rc=$?
head -8 gpurun_out/dbg5/where_sync.txt
CWDM_V5=2 CWDM_V5_ONLY=0 timeout -k 10 120 python -u tools/dbg_trace.py where 16 16 32 > gpurun_out/dbg5/where2.txt 2>&1; echo rc=$?
head -3 gpurun_out/dbg5/where2.txt
