set -o pipefail
o=gpurun_out/p3; mkdir -p $o
B="python3 bench.py --dtype bf16 --extra-dtypes= --no-extras --no-cpu-baseline --no-iou --steps 20 --warmup 5 --retune"
UNET_BF16_NORM=1 timeout -k 10 300 $B --tuning-report $o/tun_norm1.txt > $o/b_norm1.json 2> $o/b_norm1.err || exit 3
python3 - $o/b_norm1.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("bf16 norm=1", d["value"], d["ms_per_step"], {k: v["ms"] for k, v in d["kernels"].items()})
PY
timeout -k 10 1000 bash tools/prof_all.sh $o r03 "fp32 bf16" 1 > $o/prof.log 2>&1; echo prof rc=$?; tail -5 $o/prof.log
