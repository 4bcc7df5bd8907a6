"""Summarise rocprofv3 --pmc passes of bench.py per kernel family.

    python tools/pmc_report.py gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 gpurun_out/pmc4
    python tools/pmc_report.py --json profiles/pmc_traffic.json 63 gpurun_out/pmc3 gpurun_out/pmc4

Per kernel name (summed over the dispatches of the last profiled step):
effective clock = GRBM_GUI_ACTIVE / 8 XCDs / time; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES
/ (256 CUs x 4 SIMDs x clocks); HBM bytes = 2 x FETCH_SIZE (gfx950 reports half
of a wide coalesced read, MI355X_MICROARCH.md §HBM) + WRITE_SIZE, in KiB units.
"""
import collections
import csv
import json
import sys


def load(d):
    rows = list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))
    out = collections.defaultdict(dict)
    for r in rows:
        k = int(r["Dispatch_Id"])
        out[k][r["Counter_Name"]] = float(r["Counter_Value"])
        out[k]["name"] = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("unet::", "")
        out[k]["dur"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return out


def last_step(d):
    ids = sorted(d)
    starts = [i for i in ids if "conv_first_fwd" in d[i]["name"]]
    lo = starts[-1]
    return [i for i in ids if i >= lo]


def family(name):
    """Kernel family of a dispatch, matching bench.py's timing classes: the
    implicit-GEMM conv family (every igemm / halo conv / wgrad / Winograd kernel,
    the split-K epilogue and the accumulator fills its launch sites run) and the
    stage-1 kernels (inc.c0
    forward and its fused BN0-backward weight gradient + slab reduction)."""
    if "conv_first" in name or "reduce_slabs" in name:
        return "stage1"
    if ("igemm" in name or "conv3" in name or "splitk_epi" in name or "wgrad" in name or "wino" in name or
            "fillBuffer" in name):
        return "conv"  # Winograd transforms / point GEMMs and the zeroing of its wgrad accumulators included
    return "other"


def traffic(paths, sites):
    """HBM bytes (2 x FETCH_SIZE + WRITE_SIZE, KiB units) of the last profiled
    step per kernel family: per step, and for the conv family per GEMM launch
    site (bench.py's roofline.launches_per_step)."""
    tot, launches = collections.Counter(), collections.Counter()
    for path in paths:
        d = load(path)
        for i in last_step(d):
            f = family(d[i]["name"])
            if "FETCH_SIZE" in d[i]:
                tot[f] += 2 * d[i]["FETCH_SIZE"] * 1024
                launches[f] += 1
            if "WRITE_SIZE" in d[i]:
                tot[f] += d[i]["WRITE_SIZE"] * 1024
    out = {f: {"bytes_per_step": tot[f], "dispatches": launches[f]} for f in launches}
    if "conv" in out:
        out["conv"]["bytes_per_launch"] = tot["conv"] / sites
        out["conv"]["launch_sites"] = sites
    return out


def main():
    if sys.argv[1] == "--json":  # --json out.json SITES pmc_dir...
        out, sites, paths = sys.argv[2], int(sys.argv[3]), sys.argv[4:]
        json.dump({"source": " ".join(paths), "correction": "2*FETCH_SIZE + WRITE_SIZE (gfx950)",
                   "families": traffic(paths, sites)}, open(out, "w"), indent=1)
        return
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for path in sys.argv[1:]:
        d = load(path)
        for i in last_step(d):
            a = agg[d[i]["name"]]
            for k, v in d[i].items():
                if k not in ("name", "dur"):
                    a[k] += v
            a[f"dur@{path}"] += d[i]["dur"]
    print(f"{'kernel':34s} {'ms':>7s} {'clk GHz':>8s} {'MFMA%':>6s} {'wait%':>6s} {'LDSconf':>8s} {'HBM GB':>7s} {'GB/s':>7s}")
    for name, a in sorted(agg.items(), key=lambda kv: -max(v for k, v in kv[1].items() if k.startswith("dur@"))):
        durs = [v for k, v in a.items() if k.startswith("dur@")]
        t = max(durs) * 1e-9
        if t < 50e-6:
            continue
        clk = a.get("GRBM_GUI_ACTIVE", 0) / 8 / t / 1e9 if t else 0
        mfma = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (1024 * clk * 1e9 * t) * 100 if clk else 0
        wait = a.get("SQ_WAIT_ANY", 0) / max(a.get("SQ_WAVE_CYCLES", 1), 1) * 100
        hbm = (2 * a.get("FETCH_SIZE", 0) + a.get("WRITE_SIZE", 0)) * 1024 / 1e9
        print(f"{name[:34]:34s} {t * 1e3:7.2f} {clk:8.2f} {mfma:6.1f} {wait:6.1f} {a.get('SQ_LDS_BANK_CONFLICT', 0):8.2e} "
              f"{hbm:7.2f} {hbm / t:7.0f}")


if __name__ == "__main__":
    main()
