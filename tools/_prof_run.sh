set -o pipefail
o=gpurun_out/p5; mkdir -p $o
timeout -k 10 1000 bash tools/prof_all.sh $o r03 "fp32 bf16" 1 > $o/prof.log 2>&1; echo prof rc=$?; tail -4 $o/prof.log
