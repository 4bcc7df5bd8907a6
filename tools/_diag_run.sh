set -o pipefail
o=gpurun_out/g9; mkdir -p $o
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider "tests/test_gpu_model.py::test_train_step_gemm_variants_vs_oracle[tile73]" "tests/test_gpu_model.py::test_train_step_gemm_variants_vs_oracle[tile72]" > $o/t73.log 2>&1; rc=$?; tail -2 $o/t73.log; [ $rc -le 1 ] || exit $rc
B="python3 bench.py --retune --extra-dtypes= --no-extras --no-cpu-baseline --no-iou --steps 20 --warmup 5"
UNET_WINO4_FWD_MIN_CG=0 UNET_TUNE_VERBOSE=1 timeout -k 10 300 $B --tuning-report $o/tun_m0.txt > $o/b_m0.json 2> $o/b_m0.err || exit 4
UNET_TUNE_VERBOSE=1 timeout -k 10 300 $B --tuning-report $o/tun_def.txt > $o/b_def.json 2> $o/b_def.err || exit 5
python3 - $o/b_m0.json $o/b_def.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], {k: v["ms"] for k, v in d["kernels"].items()})
PY
