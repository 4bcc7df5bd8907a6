#!/bin/bash
# Kernel traces of the eager and the hipGraph bench step (same dtype, same
# tuning database), reduced by tools/graph_trace.py, with
# the weight gradients on the side stream (default) and serialised on the
# caller's stream (UNET_CONCURRENT=0: a graph without cross-queue edges).
#   tools/graph_trace.sh <outdir> [dtype]
set -o pipefail
o=${1:-gpurun_out/gtr}; dt=${2:-bf16}; mkdir -p $o
export TMPDIR=/tmp
B="bench.py --full-stdout --dtype $dt --extra-dtypes= --no-extras --no-cpu-baseline --no-iou --steps 8 --warmup 4"
for g in eager graph eager_serial graph_serial; do
  flag=""; case $g in graph*) flag="--graph";; esac
  conc=1; case $g in *serial) conc=0;; esac
  UNET_CONCURRENT=$conc timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $o/raw_$g -o run -- python3 $B $flag > $o/$g.json 2> $o/$g.err || { echo "$g trace rc=$?"; tail -5 $o/$g.err; exit 2; }
done
python3 tools/graph_trace.py $o/raw_eager $o/raw_graph 3 > $o/graph_trace.txt &&
python3 tools/graph_trace.py $o/raw_eager_serial $o/raw_graph_serial 3 > $o/graph_serial_trace.txt &&
rm -rf $o/raw_eager $o/raw_graph $o/raw_eager_serial $o/raw_graph_serial
for g in eager graph eager_serial graph_serial; do echo "$g: $(tail -c 400 $o/$g.json | grep -o '"value": [0-9.]*' | head -1)"; done
cat $o/graph_trace.txt $o/graph_serial_trace.txt
