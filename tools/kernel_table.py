"""Median duration per (kernel instantiation, grid) of a rocprofv3
--kernel-trace CSV: isolates the GEMM kernel of each variant in a
tools/conv_bench.py run (whose host timing also covers the per-op entry
point's repacks and conversions).

    python tools/kernel_table.py gpurun_out/cb_fwd/run_kernel_trace.csv [--match conv3] [--flops-file shapes]
"""
import argparse
import collections
import csv
import re
import statistics


def short(name):
    name = name.replace("void ", "").replace("unet::", "")
    name = re.sub(r"\(.*$", "", name)
    return name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default="conv3|igemm")
    args = ap.parse_args()
    groups = collections.OrderedDict()
    for r in csv.DictReader(open(args.trace)):
        nm = short(r["Kernel_Name"])
        if not re.search(args.match, nm):
            continue
        key = (nm, int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
        groups.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for (nm, gx, gy, gz), ds in groups.items():
        print(f"{nm:60s} grid {gx:8d}x{gy:4d}x{gz:2d}  n={len(ds):3d}  median {statistics.median(ds):9.1f} us")


if __name__ == "__main__":
    main()
