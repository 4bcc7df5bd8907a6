#!/bin/bash
# The round's profile set, summarised on the GPU box so only small files come
# back: per precision the rocprofv3 kernel trace + stats and the PMC passes of
# tools/prof_bench.sh, reduced by tools/pmc_report.py (per-kernel summary and
# the per-launch-site traffic JSON bench.py reads), then a 50-step kernel trace
# of the default bench reduced by tools/trace_check.py.  The kernel choices of
# every profiled pass come from one plain bench run per precision through the
# tuning database (UNET_TUNE_DB), so the counters describe the bench's kernels.
# Raw trace directories are deleted after reduction.
#   tools/prof_all.sh <outdir> <round tag, e.g. r02> ["fp32 bf16"] [trace: 1 / 0]
set -o pipefail
out=$1; tag=$2; dts=${3:-"fp32 bf16"}; do_trace=${4:-1}
export TMPDIR=/tmp
mkdir -p "$out"
for dt in $dts; do
  raw="$out/raw_$dt"
  extra=""; [ "$dt" = bf16 ] && extra="--dtype bf16"
  # tune once in a plain (unprofiled) bench run; every profiled pass replays
  # those kernel choices from the tuning database (UNET_TUNE_DB)
  export UNET_TUNE_DB="$out/tune_$dt.db"
  rm -f "$UNET_TUNE_DB"
  echo "== tune $dt"
  timeout -k 10 300 python3 bench.py --full-stdout --no-cpu-baseline --no-iou --no-extras --no-peaks --extra-dtypes= --steps 20 --warmup 5 $extra \
    > "$out/tuned_bench_$dt.json" 2> "$out/tuned_bench_$dt.err" || { echo "tune failed rc=$?"; exit 1; }
  bash tools/prof_bench.sh "$raw" $extra || exit 1
  sfx=""; [ "$dt" = bf16 ] && sfx="_bf16"
  python3 tools/pmc_report.py "$raw/pmc1" "$raw/pmc2" "$raw/pmc3" "$raw/pmc4" > "$out/${tag}_pmc_summary_$dt.txt" || exit 1
  python3 tools/pmc_report.py --json "$out/pmc_traffic$sfx.json" 63 "$raw/pmc3" "$raw/pmc4" || exit 1
  cp "$raw/trace/run_kernel_stats.csv" "$out/${tag}_rocprof_kernel_stats_$dt.csv" || exit 1
  python3 tools/step_kernels.py "$raw/trace/run_kernel_trace.csv" --top 40 > "$out/${tag}_step_kernels_$dt.txt" || exit 1
  rm -rf "$raw"
done
[ "$do_trace" = 1 ] || { echo done; exit 0; }
echo "== trace 50 steps"
export UNET_TUNE_DB="$out/tune_fp32.db"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$out/raw_tr" -o run -- python3 bench.py --full-stdout --steps 50 --warmup 10 --no-extras --no-peaks \
  --no-cpu-baseline --no-iou --extra-dtypes= > "$out/tr_bench.json" 2> "$out/tr_bench.err" || { echo "trace failed rc=$?"; tail -5 "$out/tr_bench.err"; exit 1; }
python3 tools/trace_check.py "$out/raw_tr" 10 50 "$out/tr_bench.json" > "$out/${tag}_trace_check.txt" || exit 1
rm -rf "$out/raw_tr"
echo done
