#!/bin/bash
# A/B timing runs of the bench under environment switches (kernel ablations,
# grid knobs), one process per setting, replaying one tuning database so that
# every run times the same kernel mix:
#   tools/ablate.sh <outdir> <tune_db> <dtype> "<VAR=val ...>" ["<VAR=val ...>" ...]
# Prints one line per setting: step ms and the per-class kernel ms.
out=$1; db=$2; dt=$3; shift 3
mkdir -p "$out"
i=0
for setting in "$@"; do
  i=$((i + 1))
  env $setting timeout -k 10 200 python3 bench.py --full-stdout --dtype "$dt" --tune-db "$db" --extra-dtypes= --no-extras \
    --no-cpu-baseline --no-iou --steps 5 --warmup 2 > "$out/ab$i.json" 2> "$out/ab$i.err" || { echo "failed: $setting"; exit 2; }
  python3 - "$out/ab$i.json" "$setting" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = {n: v["ms"] for n, v in d["kernels"].items()}
print(f"{sys.argv[2]:40s} step {d['ms_per_step']:.3f} ms | " + " ".join(f"{n} {v:.3f}" for n, v in k.items()), flush=True)
PY
done
