"""Per-kernel time of one train step from a rocprofv3 --kernel-trace CSV of a
bench.py run: the step is cut at k_conv_first_fwd (the first kernel of every
step); by default the last one, which is the bench's serial timing step
(weight-gradient side stream serialised), so durations do not overlap.

    python tools/step_kernels.py gpurun_out/tr/run_kernel_trace.csv [--step -1] [--top 30] [--grids]
"""
import argparse
import collections
import csv
import re


def short(name):
    name = name.replace("void ", "").replace("unet::", "")
    return re.sub(r"\(.*$", "", name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=-1, help="step index (python style; -1 = the serial timing step)")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--grids", action="store_true", help="list every launch of the step with its grid")
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "k_conv_first_fwd" in r["Kernel_Name"]]
    bounds = starts + [len(rows)]
    k = args.step % len(starts)
    step = rows[bounds[k]:bounds[k + 1]]
    span = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e6
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in step:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        a = agg[short(r["Kernel_Name"])]
        a[0] += 1
        a[1] += d
        if args.grids:
            print(f"{short(r['Kernel_Name'])[:60]:60s} grid {r['Grid_Size_X']:>9s} x {r['Grid_Size_Y']:>4s} x "
                  f"{r['Grid_Size_Z']:>3s} {d * 1e3:9.1f} us")
    print(f"step {k} of {len(starts)}: span {span:.3f} ms, kernel sum {sum(v[1] for v in agg.values()):.3f} ms")
    for name, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:args.top]:
        print(f"{ms:8.3f} ms {n:4d}  {name}")


if __name__ == "__main__":
    main()
