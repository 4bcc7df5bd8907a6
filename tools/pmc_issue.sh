# Issue mix per kernel of one profiled bench step (fp32 and bf16): one
# rocprofv3 --pmc pass each (8 SQ counters + GRBM + one TA counter), summarised
# by tools/pmc_issue.py.  Usage: bash tools/pmc_issue.sh <outdir>
set -o pipefail
export TMPDIR=/tmp
o=$1; mkdir -p $o
B="bench.py --full-stdout --no-cpu-baseline --no-iou --no-extras --no-peaks --extra-dtypes= --steps 2 --warmup 1"
C="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_WAIT_ANY TA_TA_BUSY_sum"
for dt in fp32 bf16; do
  timeout -s KILL 240 rocprofv3 --pmc $C -f csv -d $o/$dt -o run -- python3 $B --dtype $dt > $o/$dt.log 2>&1 || { echo $dt rc=$?; tail -5 $o/$dt.log; exit 3; }
  python3 tools/pmc_issue.py $o/$dt > $o/issue_$dt.txt || exit 3
  rm -rf $o/$dt
done
echo done
