#!/bin/bash
# head kernels: tests (optional -k), conv_bench (both generations) + head2 stamps
set -e -o pipefail
T=${1:-head}; K=${2:-}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
for g in 1; do
  CWDM_HEAD2=$g timeout -k 10 200 python -u tools/conv_bench.py --only L0_64_8 2>/dev/null > $O/cb_head2_$g.txt
  echo "== CWDM_HEAD2=$g"; cat $O/cb_head2_$g.txt
done
for c in L0_64_8_out L0_64_8_out_nogn; do
  CWDM_HEAD2=1 CWDM_LIB=ablib/libcwdm_stamps.so CWDM_ALLOW_STALE_LIB=1 timeout -k 10 120 python -u tools/head_stamps.py $c 2>/dev/null > $O/st_$c.txt
  cat $O/st_$c.txt
done
CWDM_LIB=ablib/libcwdm_stamps.so CWDM_ALLOW_STALE_LIB=1 timeout -k 10 200 python -u tools/head_step_stamps.py 2>&1 | grep -v amdgpu.ids > $O/st_step.txt
cat $O/st_step.txt
