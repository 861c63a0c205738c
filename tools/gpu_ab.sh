# A/B bench: alternating runs of bench.py with an env switch ($1=VAR, default CWDM_SKIP_FUSE)
set -o pipefail
V=${1:-CWDM_SKIP_FUSE}
for i in 1 2; do
  for val in 1 0; do
    env $V=$val timeout -k 10 200 python bench.py --steps 20 --warmup 3 > gpurun_out/ab.log 2>&1 || exit 1
    echo "$V=$val $(python -c "import json;d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]);print(d['value'])")"
  done
done
