set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_model.py -k "tile70 or segmented or trainer_bench" > gpurun_out/t_wino.log 2>&1; echo "wino tests rc=$?"; grep -E "PASS|FAIL|rror" gpurun_out/t_wino.log | head -20
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/pw -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --extra-dtypes= --no-iou > gpurun_out/pw.log 2>&1 || exit 1
timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --extra-dtypes= --no-iou --tuning-report gpurun_out/tuning_fp32.txt > gpurun_out/bench_w.log 2>&1 || exit 1
echo done
