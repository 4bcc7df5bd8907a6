#!/bin/bash
# rocprofv3 passes of one bench.py --full-stdout configuration (one precision, 2 timed steps
# after 1 warm-up, then the bench's serial timing step = the profiled step):
# kernel trace + stats, then one PMC pass per counter group (rocprofv3 does not
# split counters over passes; FETCH_SIZE and WRITE_SIZE cannot share one).
# Each pass under its own time limit; stop at the first failure.
#   tools/prof_bench.sh <outdir> <bench args...>
set -o pipefail
out=$1; shift
export TMPDIR=/tmp
mkdir -p "$out"
B="bench.py --full-stdout --no-cpu-baseline --no-iou --no-extras --no-peaks --extra-dtypes= --steps 2 --warmup 1"
run() { echo "== $1"; n=$1; shift; timeout -k 10 240 "$@" > "$out/$n.log" 2>&1 || { echo "failed rc=$?"; tail -5 "$out/$n.log"; exit 1; }; }
run trace rocprofv3 --kernel-trace --stats -f csv -d "$out/trace" -o run -- python3 $B "$@"
run pmc1 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES -f csv -d "$out/pmc1" -o run -- python3 $B "$@"
run pmc2 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -f csv -d "$out/pmc2" -o run -- python3 $B "$@"
run pmc3 rocprofv3 --pmc FETCH_SIZE -f csv -d "$out/pmc3" -o run -- python3 $B "$@"
run pmc4 rocprofv3 --pmc WRITE_SIZE -f csv -d "$out/pmc4" -o run -- python3 $B "$@"
echo done
