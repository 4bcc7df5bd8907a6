set -o pipefail
o=gpurun_out/g12; mkdir -p $o
P="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -rA -s"
T="tests/test_gpu_fullsize.py::test_fp32_512_every_logit_and_gradient_vs_reference_fp64 tests/test_gpu_model.py::test_sgd_trajectory_vs_reference_fixture tests/test_gpu_model.py::test_hela_train_step_real_data tests/test_gpu_fullsize.py::test_c3_572_train_step_vs_reference"
B="python3 bench.py --retune --extra-dtypes= --no-extras --no-cpu-baseline --no-iou --steps 20 --warmup 5"
for cfg in "UNET_WINO4_FWD_MIN_CG=128" "UNET_WINO4_FWD_MIN_CG=256 UNET_WINO4_FWD_SMALL_CG=64" "UNET_WINO4_FWD_MIN_CG=0"; do
  tag=$(echo $cfg | tr ' =' '__')
  env UNET_TEST_TUNE_DB= $cfg timeout -k 10 400 $P $T > $o/t_$tag.log 2>&1; echo "$cfg tests rc=$?"
  grep -E "every element|Max relative|AssertionError: \(" $o/t_$tag.log | head -4
  env $cfg timeout -k 10 300 $B > $o/b_$tag.json 2> $o/b_$tag.err || exit 5
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" $o/b_$tag.json
done
