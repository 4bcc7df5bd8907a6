"""Evidence for the data-parallel backward schedule on one GPU (VERDICT r02
item 6): the Trainer with a process group (gloo, world size 1, so every
collective is a no-op but the schedule is the DP one: 9 segmented backward
calls with the side-stream join deferred, the per-bucket reduce hook, one join
before SGD) runs a few steps; under

    rocprofv3 --kernel-trace -f csv -d <dir> -o run -- python3 tools/dp_overlap_trace.py

the kernel trace shows the weight-gradient kernels of segment s (side stream,
its own HSA queue) running while the input-gradient chain of the later
segments (the caller's queue) proceeds.  `--report <dir>` reduces the trace of
the last step to the busy time of each queue and the time both are busy.
"""
import argparse
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "unet-segmentation_amd")]


def run(steps):
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    dist.init_process_group("gloo", rank=0, world_size=1)
    from bench import init_weights, synthetic_batch
    from unet_amd import UNet
    from unet_amd.train import Trainer
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = UNet(1, 2)
    m.apply(init_weights)
    m = m.to(dev).train()
    tr = Trainer(m, 8, 512, 512, process_group=dist.group.WORLD, overlap=True)
    x, t, w = synthetic_batch(8, 512, tr.out_hw[0], dev, 1234)
    for _ in range(steps):
        tr.step(x, t, w)
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print("done", steps, "steps")


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def measure(u):
    return sum(b - a for a, b in u)


def intersect(u, v):
    i = j = 0
    tot = 0
    while i < len(u) and j < len(v):
        a, b = max(u[i][0], v[j][0]), min(u[i][1], v[j][1])
        if a < b:
            tot += b - a
        if u[i][1] < v[j][1]:
            i += 1
        else:
            j += 1
    return tot


def report(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "k_conv_first_fwd" in r["Kernel_Name"]]
    step = rows[starts[-1]:]
    qkey = "Queue_Id" if "Queue_Id" in step[0] else "Stream_Id"
    by_q = {}
    for r in step:
        by_q.setdefault(r[qkey], []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    print(f"trace {f}: last step, {len(step)} kernels on {len(by_q)} queues ({qkey})")
    us = {q: union([(a, b) for a, b, _ in v]) for q, v in by_q.items()}
    qs = sorted(us, key=lambda q: -len(by_q[q]))
    t0 = min(a for a, _, _ in sum(by_q.values(), []))
    t1 = max(b for _, b, _ in sum(by_q.values(), []))
    print(f"step span {(t1 - t0) / 1e6:.3f} ms")
    for q in qs:
        names = {}
        for _, _, n in by_q[q]:
            k = n.split("(")[0].replace("void ", "").replace("unet::", "").split("<")[0]
            names[k] = names.get(k, 0) + 1
        top = ", ".join(f"{k} x{c}" for k, c in sorted(names.items(), key=lambda kv: -kv[1])[:6])
        print(f"queue {q}: {len(by_q[q])} kernels, busy {measure(us[q]) / 1e6:.3f} ms ({top})")
    if len(qs) >= 2:
        both = intersect(us[qs[0]], us[qs[1]])
        print(f"both queues busy (weight gradients overlapping the input-gradient chain): {both / 1e6:.3f} ms")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--report", default=None)
    a = ap.parse_args()
    if a.report:
        report(a.report)
    else:
        run(a.steps)
