"""Why is whole-step hipGraph replay slower than eager launches?  (VERDICT r03
item 8.)  Reduces two `rocprofv3 --kernel-trace` runs of bench.py -- eager and
--graph, same dtype, same tuning database -- to per-step timelines:

    python tools/graph_trace.py <eager trace dir> <graph trace dir> [steps]

Per run, over the last `steps` steps (a step opens at each k_conv_first_fwd):
step span, kernel count, the union of kernel busy time, idle time between
kernels (gaps on the union timeline) and its largest gaps with the kernels on
either side, per-queue busy time and how much of the second queue's work ran
concurrently with the first's, and per-kernel-name duration sums (the same
kernels slower under replay point at the hardware queues / co-scheduling, not
at launch overhead).
"""
import collections
import csv
import glob
import os
import sys


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("unet::", "")
            q = r.get("Queue_Id", r.get("Stream_Id", "0"))
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, q))
    rows.sort()
    return rows


def steps_of(rows, n):
    opens = [i for i, r in enumerate(rows) if r[2].startswith("k_conv_first_fwd")]
    # the bench's last forward is its extra event-timed (serial) step: drop it
    opens = opens[:-1]
    out = []
    for a, b in zip(opens[-n - 1:-1], opens[-n:]):
        out.append(rows[a:b])
    return out


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e, name, _ in sorted(iv):
        if cur_e is None:
            cur_s, cur_e, last = s, e, name
            continue
        if s > cur_e:
            tot += cur_e - cur_s
            gaps.append((s - cur_e, last, name))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        last = name if e >= cur_e else last
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot, gaps


def report(tag, steps):
    print(f"== {tag}: {len(steps)} steps")
    names = collections.Counter()
    for st in steps:
        span = st[-1][1] - st[0][0]
        busy, gaps = union(st)
        byq = collections.defaultdict(list)
        for r in st:
            byq[r[3]].append(r)
        qb = {q: union(v)[0] for q, v in byq.items()}
        qs = sorted(byq, key=lambda q: -qb[q])
        conc = ""
        if len(qs) > 1:
            both = qb[qs[0]] + qb[qs[1]] - union(byq[qs[0]] + byq[qs[1]])[0]
            conc = f", queue {qs[1]} busy {qb[qs[1]] / 1e6:.2f} ms of which concurrent with queue {qs[0]}: {both / 1e6:.2f} ms"
        print(f"  span {span / 1e6:.3f} ms, {len(st)} kernels, busy union {busy / 1e6:.3f} ms, idle {sum(g[0] for g in gaps) / 1e6:.3f} ms "
              f"in {len(gaps)} gaps; queues {len(byq)}: " + ", ".join(f"{q}:{qb[q] / 1e6:.2f}" for q in qs) + conc)
        for g, a, b in sorted(gaps, reverse=True)[:4]:
            print(f"     gap {g / 1e3:7.1f} us  {a[:40]} -> {b[:40]}")
        for s, e, n, _ in st:
            names[n] += e - s
    print("  per-kernel duration per step (ms):")
    for n, t in names.most_common(12):
        print(f"     {t / len(steps) / 1e6:7.3f}  {n[:70]}")
    return names


def main():
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    a = report("eager", steps_of(load(sys.argv[1]), k))
    b = report("graph", steps_of(load(sys.argv[2]), k))
    print("== largest per-kernel differences graph - eager (ms per step):")
    diff = {n: (b.get(n, 0) - a.get(n, 0)) / k / 1e6 for n in set(a) | set(b)}
    for n, d in sorted(diff.items(), key=lambda x: -abs(x[1]))[:12]:
        print(f"     {d:+7.3f}  {n[:70]}")


if __name__ == "__main__":
    main()
