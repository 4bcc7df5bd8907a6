set -o pipefail
o=gpurun_out/gab; mkdir -p $o
B="python3 bench.py --full-stdout --extra-dtypes= --no-extras --no-cpu-baseline --no-iou --steps 20 --warmup 5"
for dt in bf16 fp32; do
  for g in "" "--graph" ""; do
    timeout -k 10 300 $B --dtype $dt $g > $o/b_${dt}${g}.json 2> $o/b_${dt}${g}.err || { echo fail $dt $g; exit 2; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['mean_ms_per_step'])" $o/b_${dt}${g}.json "$dt $g"
  done
done
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
