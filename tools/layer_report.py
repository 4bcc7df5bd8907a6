"""Per-layer report from a rocprofv3 kernel trace of bench.py.

Maps the k_igemm / k_wgrad dispatches of one training step onto the U-Net
layers (the plan's fixed launch order) and prints time and TFLOP/s per layer.
    python tools/layer_report.py gpurun_out/prof2/run_kernel_trace.csv [batch] [size]
"""
import csv
import sys


def geometry(n=8, h=512):
    chans = [64, 128, 256, 512, 1024]
    L = []
    hh, cprev = h, 1
    for b in range(5):
        if b:
            hh //= 2
        for j in range(2):
            ci = cprev if j == 0 else chans[b]
            L.append(dict(ci=ci, co=chans[b], hi=hh, ho=hh - 2))
            hh -= 2
        cprev = chans[b]
    T = []
    for k in range(4):
        prev = L[9 + 2 * k]
        T.append(dict(ci=prev["co"], co=prev["co"] // 2, h=prev["ho"]))
        enc = L[7 - 2 * k]
        th = 2 * prev["ho"]
        for j in range(2):
            ci = enc["co"] + prev["co"] // 2 if j == 0 else prev["co"] // 2
            L.append(dict(ci=ci, co=prev["co"] // 2, hi=th, ho=th - 2))
            th -= 2
    names = ["inc.c0", "inc.c1"] + [f"down{b}.c{j}" for b in range(1, 5) for j in range(2)] + \
            [f"up{k}.c{j}" for k in range(1, 5) for j in range(2)]
    seq = []
    cf = lambda l: 2.0 * n * l["ho"] ** 2 * l["co"] * l["ci"] * 9
    tf = lambda t: 2.0 * n * t["h"] ** 2 * t["ci"] * t["co"] * 4
    for l in range(1, 18):
        if l >= 10 and l % 2 == 0:
            seq.append((f"up{(l - 10) // 2 + 1}.convT fwd", tf(T[(l - 10) // 2])))
        seq.append((f"{names[l]} fwd", cf(L[l])))
    for l in range(17, 0, -1):
        seq.append((f"{names[l]} wgrad", cf(L[l])))
        seq.append((f"{names[l]} dgrad", cf(L[l])))
        if l >= 10 and l % 2 == 0:
            k = (l - 10) // 2
            seq.append((f"up{k + 1}.convT wgrad", tf(T[k])))
            seq.append((f"up{k + 1}.convT dgrad", tf(T[k])))
    return seq


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    h = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "conv_first_fwd" in r["Kernel_Name"]]
    # the last step of bench.py is its serial timing step (no side stream)
    step = rows[starts[-1]:]
    conv = [r for r in step if any(k in r["Kernel_Name"] for k in ("k_igemm", "k_wgrad", "k_conv3"))]
    seq = geometry(n, h)
    assert len(conv) == len(seq), (len(conv), len(seq))
    tot_t = tot_f = 0.0
    print(f"{'layer':24s} {'kernel':26s} {'blocks':>7s} {'us':>8s} {'TF/s':>7s}")
    for (name, fl), r in zip(seq, conv):
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        gx = int(r["Grid_Size_X"]) // int(r.get("Workgroup_Size_X", 256)) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        kn = r["Kernel_Name"].split("(")[0].replace("void unet::", "")
        tot_t += us
        tot_f += fl
        print(f"{name:24s} {kn:26s} {gx:7d} {us:8.1f} {fl / us / 1e6:7.1f}")
    all_us = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e3
    print(f"conv total {tot_t / 1e3:.2f} ms, {tot_f / tot_t / 1e6:.1f} TF/s; step span {all_us / 1e3:.2f} ms")
    other = {}
    for r in step:
        if r in conv:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void unet::", "").replace("unet::", "")
        other[k] = other.get(k, 0.0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for k, v in sorted(other.items(), key=lambda kv: -kv[1]):
        print(f"  {k:40s} {v:8.1f} us")


if __name__ == "__main__":
    main()
