#!/bin/bash
# rocprofv3 kernel trace of the DP backward schedule on one GPU and its reduction
set -o pipefail
o=${1:-gpurun_out/ovl}; mkdir -p $o
export TMPDIR=/tmp UNET_TUNE_DB=$o/tune_db.txt
cp profiles/tune_db.txt $o/tune_db.txt
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $o/raw -o run -- python3 tools/dp_overlap_trace.py --steps 4 > $o/run.log 2>&1 || { echo trace rc=$?; tail -5 $o/run.log; exit 2; }
python3 tools/dp_overlap_trace.py --report $o/raw > $o/overlap.txt && rm -rf $o/raw
cat $o/overlap.txt
