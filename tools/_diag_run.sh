set -o pipefail
o=gpurun_out/g6; mkdir -p $o
T="tests/test_gpu_fullsize.py::test_fp32_512_every_logit_and_gradient_vs_reference_fp64 tests/test_gpu_model.py::test_sgd_trajectory_vs_reference_fixture"
P="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -rA -s"
timeout -k 10 300 $P tests/test_gpu_fullsize.py::test_trainer_bf16_batch8_512_vs_reference "tests/test_gpu_fullsize.py::test_c3_572_train_step_vs_reference" > $o/t_bf16.log 2>&1; echo bf16 rc=$?
B="python bench.py --retune --extra-dtypes= --no-extras --no-cpu-baseline --no-iou --steps 20 --warmup 5"
for m in 128 256 512; do
  UNET_TEST_TUNE_DB= UNET_WINO4_FWD_MIN_CG=$m timeout -k 10 300 $P $T > $o/t_m$m.log 2>&1; echo m$m tests rc=$?
  UNET_WINO4_FWD_MIN_CG=$m timeout -k 10 300 $B > $o/b_m$m.json 2> $o/b_m$m.err || exit 5
done
python3 - $o/b_m*.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], {k: v["ms"] for k, v in d["kernels"].items()})
PY
