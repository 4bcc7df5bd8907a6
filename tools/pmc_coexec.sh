set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5h; mkdir -p $o
B="bench.py --full-stdout --no-cpu-baseline --no-iou --no-extras --no-peaks --extra-dtypes= --steps 2 --warmup 1"
C="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
timeout -s KILL 240 rocprofv3 --pmc $C -f csv -d $o/fp32 -o run -- python3 $B > $o/fp32.log 2>&1 || { echo fp32 rc=$?; tail -5 $o/fp32.log; exit 3; }
python3 tools/pmc_coexec.py $o/fp32 > $o/coexec_fp32.txt || exit 3
timeout -s KILL 240 rocprofv3 --pmc $C -f csv -d $o/bf16 -o run -- python3 $B --dtype bf16 > $o/bf16.log 2>&1 || { echo bf16 rc=$?; tail -5 $o/bf16.log; exit 3; }
python3 tools/pmc_coexec.py $o/bf16 > $o/coexec_bf16.txt || exit 3
rm -rf $o/fp32 $o/bf16
echo done
