set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/cb_fwd -o run -- python3 tools/conv_bench.py --a16 --reps 5 > gpurun_out/cb_fwd.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/cb_dgrad -o run -- python3 tools/conv_bench.py --a16 --dgrad --reps 5 > gpurun_out/cb_dgrad.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1; echo "tests rc=$?"; tail -5 gpurun_out/t_all.log
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit 1
echo done
