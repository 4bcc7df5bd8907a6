set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -f csv -d gpurun_out/cbp1 -o run -- python3 tools/conv_bench.py --a16 --reps 2 --shapes inc.c1,down1.c1,down3.c1 --variants 31,33,62,63,65 > gpurun_out/cbp1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SMEM SQ_INSTS_VMEM -f csv -d gpurun_out/cbp2 -o run -- python3 tools/conv_bench.py --a16 --reps 2 --shapes inc.c1,down1.c1,down3.c1 --variants 31,33,62,63,65 > gpurun_out/cbp2.log 2>&1 || exit 1
echo done
