"""Issue mix per kernel of the last profiled bench step (tools/pmc_issue.sh).

    python tools/pmc_issue.py <pmc dir>

Per kernel, summed over the step's dispatches; shares of SQ_WAVE_CYCLES
(wave-cycles; quad-cycle units for the ACTIVE_INST counters, hence x4):
  any / valu / lds / sca / vmem = 4 x SQ_ACTIVE_INST_* / SQ_WAVE_CYCLES
  ldswait = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES, wait = SQ_WAIT_ANY / SQ_WAVE_CYCLES
  ta% = TA_TA_BUSY_sum / (256 CUs x clocks)
"""
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_report import last_step, load  # noqa: E402


def main():
    d = load(sys.argv[1])
    agg = {}
    for i in last_step(d):
        a = agg.setdefault(d[i]["name"], {"dur": 0.0, "n": 0})
        for k, v in d[i].items():
            if k not in ("name", "dur"):
                a[k] = a.get(k, 0.0) + v
        a["dur"] += d[i]["dur"]
        a["n"] += 1
    cols = ["any", "valu", "lds", "sca", "vmem", "ldswait", "wait", "ta"]
    print(f"{'kernel':44s} {'n':>3s} {'ms':>7s} " + " ".join(f"{c + '%':>8s}" for c in cols))
    for name, a in sorted(agg.items(), key=lambda kv: -kv[1]["dur"]):
        t = a["dur"] * 1e-9
        if t < 30e-6:
            continue
        wc = max(a.get("SQ_WAVE_CYCLES", 1), 1)
        clk = a.get("GRBM_GUI_ACTIVE", 0) / 8 / t if t else 0
        v = [4 * a.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4 * a.get("SQ_ACTIVE_INST_VALU", 0) / wc,
             4 * a.get("SQ_ACTIVE_INST_LDS", 0) / wc, 4 * a.get("SQ_ACTIVE_INST_SCA", 0) / wc,
             4 * a.get("SQ_ACTIVE_INST_VMEM", 0) / wc, a.get("SQ_WAIT_INST_LDS", 0) / wc,
             a.get("SQ_WAIT_ANY", 0) / wc, a.get("TA_TA_BUSY_sum", 0) / (256 * clk * t) if clk else 0]
        print(f"{name[:44]:44s} {a['n']:3d} {t * 1e3:7.3f} " + " ".join(f"{100 * x:8.1f}" for x in v))


if __name__ == "__main__":
    main()
