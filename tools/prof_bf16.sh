#!/bin/bash
# rocprofv3 passes of one bench.py configuration: kernel trace + stats, then
# one PMC pass per counter group (rocprofv3 does not split counters over
# passes; FETCH_SIZE and WRITE_SIZE cannot share one).  Each pass under its own
# time limit; stop at the first failure.
#   tools/prof_bf16.sh <outdir> <bench args...>
set -o pipefail
out=$1; shift
export TMPDIR=/tmp
run() { echo "== $1"; shift; timeout -k 10 240 "$@" > "$out.$(date +%s%N).log" 2>&1 || { echo "failed rc=$?"; exit 1; }; }
mkdir -p "$out"
run trace rocprofv3 --kernel-trace --stats -f csv -d "$out/trace" -o run -- python3 bench.py --no-cpu-baseline "$@"
run pmc1 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES -f csv -d "$out/pmc1" -o run -- python3 bench.py --no-cpu-baseline "$@"
run pmc2 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -f csv -d "$out/pmc2" -o run -- python3 bench.py --no-cpu-baseline "$@"
run pmc3 rocprofv3 --pmc FETCH_SIZE -f csv -d "$out/pmc3" -o run -- python3 bench.py --no-cpu-baseline "$@"
run pmc4 rocprofv3 --pmc WRITE_SIZE -f csv -d "$out/pmc4" -o run -- python3 bench.py --no-cpu-baseline "$@"
echo done
