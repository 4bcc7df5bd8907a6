"""Per-step kernel times of a `rocprofv3 --kernel-trace` run of bench.py.

    rocprofv3 --kernel-trace --stats -d gpurun_out/tr -o run -- python bench.py --steps K --warmup W
    python tools/trace_check.py gpurun_out/tr W K [bench.json]

`rocprofv3 --stats` averages each kernel over every dispatch of the process,
autotuner trials included (the tuner times each candidate tile in the first
warm-up step), so its per-kernel averages are not the bench's numbers.  This
script splits the trace into steps at the `k_conv_first_fwd` dispatch that
opens every forward, keeps the K timed steps (after the W warm-up steps, before
bench.py's one extra event-timed step) and reports, per step, the implicit-GEMM
conv family (k_igemm*, k_conv3*, k_wgrad*, with and without the split-K
epilogue k_splitk_epi), the elementwise kernels and the dispatch span.  With the
bench JSON line it prints the bench's `roofline.avg_launch_ms` beside the
trace's average GEMM launch.
"""
import collections
import csv
import glob
import json
import os
import sqlite3
import sys

GEMM = ("k_igemm", "k_conv3", "k_wgrad", "k_wino", "fillBuffer")  # Winograd + its wgrad accumulator fills


def short(name):
    return name.split("(")[0].replace("void ", "").replace("unet::", "")


def load(d):
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    if not files:  # rocprofv3's default output: one rocpd SQLite database per process
        dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
        if not dbs:
            raise SystemExit(f"no *kernel_trace.csv or *.db under {d}")
        for f in dbs:
            con = sqlite3.connect(f)
            rows += [(int(s), int(e), short(n)) for s, e, n in con.execute("select start, end, name from kernels")]
        rows.sort()
        return rows
    for f in files:
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    return rows


def main():
    d, warm, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    bench = None
    if len(sys.argv) > 4:
        line = [ln for ln in open(sys.argv[4]) if ln.startswith("{")][-1]
        bench = json.loads(line)
    rows = load(d)
    opens = [i for i, r in enumerate(rows) if r[2].startswith("k_conv_first_fwd")]
    print(f"trace: {len(rows)} dispatches, {len(opens)} forward passes (expected warmup {warm} + steps {steps} + 1 timing step)")
    if len(opens) < warm + steps:
        raise SystemExit("fewer forward passes than warmup + steps")
    lo = opens[warm]
    hi = opens[warm + steps] if warm + steps < len(opens) else len(rows)
    sel = rows[lo:hi]
    per = collections.defaultdict(lambda: [0, 0])
    for s, e, n in sel:
        per[n][0] += 1
        per[n][1] += e - s
    g_n = sum(v[0] for k, v in per.items() if k.startswith(GEMM))
    g_t = sum(v[1] for k, v in per.items() if k.startswith(GEMM))
    epi_n, epi_t = per.get("k_splitk_epi", [0, 0])
    other_t = sum(v[1] for k, v in per.items() if not k.startswith(GEMM) and k != "k_splitk_epi")
    span = (sel[-1][1] - sel[0][0]) / steps
    # wall time with at least one GEMM (or its split-K epilogue) running: the
    # union of their dispatch intervals (the side stream overlaps them)
    busy, cur_s, cur_e = 0, None, None
    for s, e, n in sorted(r for r in sel if r[2].startswith(GEMM) or r[2] == "k_splitk_epi"):
        if cur_e is None or s > cur_e:
            busy += 0 if cur_e is None else cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += 0 if cur_e is None else cur_e - cur_s
    print(f"timed steps {warm}..{warm + steps - 1}: span {span / 1e6:.3f} ms/step (first dispatch to last, incl. the SGD)")
    print(f"GEMM kernels (Winograd transforms and fills included): {g_n / steps:.1f} launches/step, {g_t / steps / 1e6:.3f} ms/step, "
          f"avg {g_t / g_n / 1e6:.4f} ms/launch")
    print(f"  + split-K epilogue: {epi_n / steps:.1f} launches/step, {epi_t / steps / 1e6:.3f} ms/step; "
          f"GEMM+epilogue per GEMM launch {(g_t + epi_t) / g_n / 1e6:.4f} ms")
    print(f"other kernels: {other_t / steps / 1e6:.3f} ms/step")
    if bench:
        r = bench["roofline"]
        lps = r["launches_per_step"]
        fl = r.get("mfma_flops_per_step", r.get("flops_per_step"))  # executed MFMA flops (round 2 line)
        tr_avg = (g_t + epi_t) / steps / lps / 1e6
        print(f"bench.py (HIP events, one extra step): {lps} conv-family launches/step, "
              f"avg {r['avg_launch_ms']:.4f} ms/launch, {r['achieved']:.2f} TFLOP/s")
        print(f"trace (timed steps): GEMM+epilogue / {lps} = {tr_avg:.4f} ms/launch, "
              f"{fl / (tr_avg * lps * 1e-3) / 1e12:.2f} TFLOP/s "
              f"(ratio trace/bench {tr_avg / r['avg_launch_ms']:.3f})")
        print(f"trace (timed steps): GEMM-busy wall time {busy / steps / 1e6:.3f} ms/step (union of intervals) = "
              f"{fl / (busy / steps * 1e-9) / 1e12:.2f} TFLOP/s over the timed region")
        print(f"bench ms_per_step {bench['ms_per_step']:.3f} vs trace span {span / 1e6:.3f}")
    print("\nper kernel over the timed steps (calls/step, ms/step, avg us):")
    for k, (n, t) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"  {k:<44} {n / steps:6.1f} {t / steps / 1e6:8.3f} {t / n / 1e3:9.1f}")


if __name__ == "__main__":
    main()
