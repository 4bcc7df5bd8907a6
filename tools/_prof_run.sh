set -o pipefail
o=gpurun_out/p4; mkdir -p $o
timeout -k 10 700 bash tools/prof_all.sh $o r03 "fp32 bf16" 0 > $o/prof.log 2>&1; echo prof rc=$?; tail -3 $o/prof.log
timeout -k 10 660 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $o/gpu_tests.log 2>&1; echo tests rc=$?
tail -6 $o/gpu_tests.log
