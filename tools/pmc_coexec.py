"""VALU / MFMA co-execution of the kernels of one profiled bench step.

One rocprofv3 --pmc pass of bench.py with
  GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES
  SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES
(does the Winograd transform VALU hide under the f32 MFMAs?).

    python tools/pmc_coexec.py <pmc dir> [kernel substring ...]

Per kernel, summed over the dispatches of the last profiled step:
  MFMA%   = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x clocks)      (busy share of the MFMA pipe)
  coex%   = SQ_VALU_MFMA_COEXEC_CYCLES / SQ_VALU_MFMA_BUSY_CYCLES (MFMA-busy cycles in which a VALU op also issued)
  VALU%   = 4 x SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES               (wave-cycles spent issuing VALU; quad-cycle units)
  wait% / instwait% = SQ_WAIT_ANY / SQ_WAIT_INST_ANY over SQ_WAVE_CYCLES
"""
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_report import last_step, load  # noqa: E402


def main():
    d = load(sys.argv[1])
    want = sys.argv[2:]
    agg = {}
    for i in last_step(d):
        name = d[i]["name"]
        if want and not any(w in name for w in want):
            continue
        a = agg.setdefault(name, {"dur": 0.0, "n": 0})
        for k, v in d[i].items():
            if k not in ("name", "dur"):
                a[k] = a.get(k, 0.0) + v
        a["dur"] += d[i]["dur"]
        a["n"] += 1
    print(f"{'kernel':44s} {'n':>3s} {'ms':>7s} {'GHz':>5s} {'MFMA%':>6s} {'coex%':>6s} {'VALU%':>6s} {'wait%':>6s} "
          f"{'iwait%':>6s}")
    for name, a in sorted(agg.items(), key=lambda kv: -kv[1]["dur"]):
        t = a["dur"] * 1e-9
        if t < 30e-6:
            continue
        clk = a.get("GRBM_GUI_ACTIVE", 0) / 8 / t / 1e9 if t else 0
        busy = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
        mfma = busy / (1024 * clk * 1e9 * t) * 100 if clk else 0
        coex = a.get("SQ_VALU_MFMA_COEXEC_CYCLES", 0) / busy * 100 if busy else 0
        wc = max(a.get("SQ_WAVE_CYCLES", 1), 1)
        valu = 4 * a.get("SQ_ACTIVE_INST_VALU", 0) / wc * 100
        wait = a.get("SQ_WAIT_ANY", 0) / wc * 100
        iwait = a.get("SQ_WAIT_INST_ANY", 0) / wc * 100
        print(f"{name[:44]:44s} {a['n']:3d} {t * 1e3:7.3f} {clk:5.2f} {mfma:6.1f} {coex:6.1f} {valu:6.1f} {wait:6.1f} "
              f"{iwait:6.1f}")


if __name__ == "__main__":
    main()
