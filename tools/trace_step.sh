# Kernel trace of one timed bench step per precision (fresh autotune), reduced
# to per-kernel step times by tools/step_kernels.py.  tools/trace_step.sh <outdir>
set -o pipefail
export TMPDIR=/tmp
o=${1:-gpurun_out/g8}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $o/tr32 -o run -- python3 bench.py --full-stdout --no-cpu-baseline --no-iou --extra-dtypes= --no-extras --steps 2 --warmup 1 --retune > $o/tr32.json 2> $o/tr32.err || exit 3
python3 tools/step_kernels.py $o/tr32/run_kernel_trace.csv --top 45 > $o/step32.txt || exit 4
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $o/tr16 -o run -- python3 bench.py --full-stdout --dtype bf16 --no-cpu-baseline --no-iou --extra-dtypes= --no-extras --steps 2 --warmup 1 --retune > $o/tr16.json 2> $o/tr16.err || exit 5
python3 tools/step_kernels.py $o/tr16/run_kernel_trace.csv --top 45 > $o/step16.txt || exit 6
rm -rf $o/tr32 $o/tr16
