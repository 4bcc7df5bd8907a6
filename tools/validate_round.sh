#!/bin/bash
# Round validation on the GPU box, in the order the driver's round-end checks
# depend on: the bench with fresh autotuning writes the GEMM choices it timed to
# profiles/tune_db.txt (which the full-size tests replay), the full-size tests'
# own shapes are added to it (tools/tune_test_shapes.py), then the whole GPU
# suite runs against that database.
#   gpurun -- 'bash tools/validate_round.sh [outdir]'
set -o pipefail
o=${1:-gpurun_out/validate}; mkdir -p $o
timeout -k 10 480 python bench.py --steps 20 --warmup 5 --retune --tune-db-out profiles/tune_db.txt --tuning-report $o/tuning.txt --detail-out $o/bench_detail.json > $o/bench.json 2> $o/bench.err || { echo bench rc=$?; tail -5 $o/bench.err; exit 3; }
timeout -k 10 700 python tools/tune_test_shapes.py profiles/tune_db.txt > $o/tune_tests.log 2>&1 || { echo tune_test_shapes rc=$?; tail -5 $o/tune_tests.log; exit 3; }
cp profiles/tune_db.txt $o/tune_db.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -p no:cacheprovider -rf > $o/gpu_tests.log 2>&1; echo tests rc=$?
tail -6 $o/gpu_tests.log
