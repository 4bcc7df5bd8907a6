#!/bin/bash
# Same-box A/B of bench settings (box-to-box speed differs by up to ~8 %, so
# compare settings inside one gpurun call): one retuned bench per setting.
#   tools/ab_env.sh <outdir> <dtype> "<VAR=val ...>" ["<VAR=val ...>" ...]
set -o pipefail
o=$1; dt=$2; shift 2; mkdir -p $o
i=0
for cfg in "$@"; do
  i=$((i + 1))
  env $cfg timeout -k 10 300 python3 bench.py --full-stdout --dtype $dt --retune --extra-dtypes= --no-extras --no-cpu-baseline \
    --no-iou --steps 20 --warmup 5 > $o/ab$i.json 2> $o/ab$i.err || { echo "failed: $cfg"; exit 2; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()})" $o/ab$i.json "$cfg"
done
