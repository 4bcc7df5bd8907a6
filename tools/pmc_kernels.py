"""Per-kernel summary of rocprofv3 --pmc passes (counters summed over every
dispatch of a kernel name and grid): MFMA busy, wave wait shares and the
instruction mix per MFMA.

    python tools/pmc_kernels.py <pass dir> [<pass dir> ...]
"""
import collections
import csv
import sys


def main():
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for d in sys.argv[1:]:
        for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("unet::", "")
            key = (name, r.get("Grid_Size", "?"))
            agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
            if r["Counter_Name"] in ("SQ_WAVE_CYCLES", "SQ_INSTS_MFMA"):
                disp[key].add((d, r["Dispatch_Id"]))
                agg[key]["dur_" + d] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for (name, grid), c in sorted(agg.items()):
        mf = c.get("SQ_INSTS_MFMA", 0)
        wc = c.get("SQ_WAVE_CYCLES", 0)
        line = f"{name[:60]:60s} grid {grid:>9s}"
        gr = c.get("GRBM_GUI_ACTIVE", 0)
        if gr:
            # GRBM_GUI_ACTIVE sums the 8 XCDs' cycles; 1024 SIMDs; MFMA busy counts cycles
            line += f" mfma_busy {c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (gr / 8 * 1024) * 100:5.1f}%"
        if wc:
            line += (f" wait {c.get('SQ_WAIT_ANY', 0) / wc * 100:4.1f}% inst_wait {c.get('SQ_WAIT_INST_ANY', 0) / wc * 100:4.1f}%"
                     f" active {c.get('SQ_ACTIVE_INST_ANY', 0) / wc * 100:4.1f}%")
        if mf:
            line += (f" | per MFMA: valu {c.get('SQ_INSTS_VALU', 0) / mf:5.2f} salu {c.get('SQ_INSTS_SALU', 0) / mf:5.2f}"
                     f" lds {c.get('SQ_INSTS_LDS', 0) / mf:5.2f} vmem {c.get('SQ_INSTS_VMEM', 0) / mf:5.2f}"
                     f" | lds_conflict/active {c.get('SQ_LDS_BANK_CONFLICT', 0) / max(c.get('SQ_LDS_IDX_ACTIVE', 1), 1):5.3f}"
                     f" lds_issue_wait {c.get('SQ_WAIT_INST_LDS', 0):.3g}")
        print(line)


if __name__ == "__main__":
    main()
