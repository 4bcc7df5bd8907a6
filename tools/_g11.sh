set -o pipefail
o=${1:-gpurun_out/g11}
mkdir -p $o
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread -m gpu tests/test_gpu_model.py -k "tile73 or tile72 or heuristic or channel" > $o/t73.log 2>&1 || { tail -30 $o/t73.log; exit 3; }
tail -2 $o/t73.log
UNET_TUNE_VERBOSE=1 timeout -k 10 900 python bench.py --retune --tune-db-out $o/tune_db.txt --tuning-report $o/tuning.txt > $o/bench.json || exit 4
python3 - $o/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("fp32", d["value"], d["ms_per_step"], {k: v["ms"] for k, v in d["kernels"].items()})
b = d["bf16"]; print("bf16", b["value"], b["ms_per_step"], {k: v["ms"] for k, v in b["kernels"].items()})
PY
