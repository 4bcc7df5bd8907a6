set -o pipefail
o=gpurun_out/g3; mkdir -p $o
timeout -k 10 300 python tools/bf16_diag.py --small 2,252 > $o/small_252.txt 2>&1 || exit 3
UNET_AUTOTUNE=0 timeout -k 10 300 python tools/bf16_diag.py --small 2,252 > $o/small_252_heur.txt 2>&1 || exit 4
T="tests/test_gpu_fullsize.py::test_fp32_512_every_logit_and_gradient_vs_reference_fp64 tests/test_gpu_model.py::test_sgd_trajectory_vs_reference_fixture tests/test_gpu_fullsize.py::test_c3_572_train_step_vs_reference tests/test_gpu_pipeline.py"
P="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -rA"
timeout -k 10 400 $P $T > $o/t_default.log 2>&1; echo default rc=$?
UNET_TEST_TUNE_DB= UNET_WINO_WGRAD_MAX=4 timeout -k 10 400 $P $T > $o/t_wg4.log 2>&1; echo wg4 rc=$?
UNET_TEST_TUNE_DB= UNET_TUNE_SKIP=73 timeout -k 10 400 $P $T > $o/t_no73.log 2>&1; echo no73 rc=$?
exit 0
