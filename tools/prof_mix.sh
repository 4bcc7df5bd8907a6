#!/bin/bash
# Instruction-mix PMC passes (MFMA busy, wait shares, VALU / SALU / LDS / VMEM
# per MFMA, LDS bank conflicts) of any python command, reduced per kernel by
# tools/pmc_kernels.py.  Each pass under its own time limit.
#   tools/prof_mix.sh <outdir> <script.py> [args...]
#   e.g. tools/prof_mix.sh gpurun_out/mix bench.py --no-cpu-baseline --no-iou --extra-dtypes= --no-extras --steps 2 --warmup 1
set -o pipefail
out=$1; shift
export TMPDIR=/tmp
mkdir -p "$out"
run() { echo "== $1"; n=$1; shift; timeout -s KILL 240 "$@" > "$out/$n.log" 2>&1 || { echo "failed rc=$?"; tail -5 "$out/$n.log"; exit 1; }; }
run pa rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -f csv -d "$out/pa" -o run -- python3 "$@"
run pb rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -f csv -d "$out/pb" -o run -- python3 "$@"
python3 tools/pmc_kernels.py "$out/pa" "$out/pb" > "$out/summary.txt" || exit 1
rm -rf "$out/pa" "$out/pb"
echo done
